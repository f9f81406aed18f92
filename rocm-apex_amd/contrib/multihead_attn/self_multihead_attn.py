"""SelfMultiheadAttn (reference apex/contrib/multihead_attn/self_multihead_attn.py:26-258).

Same constructor / forward signature and parameter names as the reference (so checkpoints
load); ``impl="fast"`` runs the gfx950 flash-attention kernel, ``impl="default"`` torch math.
Unlike the reference's fast path, additive masks and biases are supported together, and
``include_norm_add`` works with every option."""
import math

import torch
from torch import nn
from torch.nn import Parameter

from ...normalization.fused_layer_norm import FusedLayerNorm
from ._core import dropout_add, self_attn


class SelfMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False, impl="fast",
                 separate_qkv_params=False, mask_additive=False):
        super().__init__()
        assert impl in ("fast", "default"), "Unsupported impl: {} !".format(impl)
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == self.embed_dim, "embed_dim must be divisible by num_heads"
        self.bias = bias
        self.include_norm_add = include_norm_add
        self.impl = impl
        self.scaling = self.head_dim ** -0.5
        self.separate_qkv_params = separate_qkv_params
        self.mask_additive = mask_additive
        if mask_additive:
            assert not include_norm_add, "additive mask not supported with layer norm"
        if separate_qkv_params:
            self.q_weight = Parameter(torch.empty(embed_dim, embed_dim))
            self.k_weight = Parameter(torch.empty(embed_dim, embed_dim))
            self.v_weight = Parameter(torch.empty(embed_dim, embed_dim))
        else:
            self.in_proj_weight = Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.out_proj_weight = Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            if separate_qkv_params:
                self.q_bias = Parameter(torch.empty(embed_dim))
                self.k_bias = Parameter(torch.empty(embed_dim))
                self.v_bias = Parameter(torch.empty(embed_dim))
            else:
                self.in_proj_bias = Parameter(torch.empty(3 * embed_dim))
            self.out_proj_bias = Parameter(torch.empty(embed_dim))
        else:
            if separate_qkv_params:
                self.register_parameter("q_bias", None)
                self.register_parameter("k_bias", None)
                self.register_parameter("v_bias", None)
            else:
                self.register_parameter("in_proj_bias", None)
            self.register_parameter("out_proj_bias", None)
        if include_norm_add:
            if impl == "fast":
                self.lyr_nrm_gamma_weights = Parameter(torch.empty(embed_dim))
                self.lyr_nrm_beta_weights = Parameter(torch.empty(embed_dim))
                self.lyr_nrm = None
            else:
                self.register_parameter("lyr_norm_gamma_weights", None)
                self.register_parameter("lyr_norm_beta_weights", None)
                self.lyr_nrm = FusedLayerNorm(embed_dim)
        self.reset_parameters()

    def reset_parameters(self):
        if self.separate_qkv_params:
            nn.init.xavier_uniform_(self.q_weight)
            nn.init.xavier_uniform_(self.k_weight)
            nn.init.xavier_uniform_(self.v_weight)
        else:
            # [3E, E] initialised like an [E, E] matrix (reference :118-121)
            nn.init.xavier_uniform_(self.in_proj_weight, gain=math.sqrt(2))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            if self.separate_qkv_params:
                for b in (self.q_bias, self.k_bias, self.v_bias):
                    nn.init.constant_(b, 0.0)
            else:
                nn.init.constant_(self.in_proj_bias, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)
        if self.include_norm_add:
            if self.impl == "fast":
                nn.init.ones_(self.lyr_nrm_gamma_weights)
                nn.init.zeros_(self.lyr_nrm_beta_weights)
            else:
                self.lyr_nrm.reset_parameters()

    def _input_weights(self):
        if not self.separate_qkv_params:
            return self.in_proj_weight, self.in_proj_bias
        h, d, e = self.num_heads, self.head_dim, self.embed_dim
        w = torch.cat([self.q_weight.view(h, 1, d, e), self.k_weight.view(h, 1, d, e),
                       self.v_weight.view(h, 1, d, e)], dim=1).reshape(3 * e, e)
        b = None
        if self.bias:
            b = torch.cat([self.q_bias.view(h, 1, d), self.k_bias.view(h, 1, d), self.v_bias.view(h, 1, d)],
                          dim=1).reshape(3 * e)
        return w, b

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, attn_mask=None,
                is_training=True):
        """query [seq, batch, embed] (self attention: key / value are ignored, as in the reference)."""
        if key_padding_mask is not None:
            assert attn_mask is None, "ERROR attn_mask and key_padding_mask should not be both defined!"
        elif attn_mask is not None:
            assert not self.mask_additive, "additive mask not supported for time mask"
        w, b = self._input_weights()
        mask = key_padding_mask if key_padding_mask is not None else attn_mask
        use_time_mask = attn_mask is not None
        if self.include_norm_add and self.impl == "fast":
            # the reference's fast_self_attn_norm_add_func: LN -> attention -> dropout + residual
            out = self_attn(use_time_mask, is_training, self.num_heads, self.scaling, query, w,
                            self.out_proj_weight, b, self.out_proj_bias, mask, self.mask_additive, self.dropout,
                            "fast", norm=(self.lyr_nrm_gamma_weights, self.lyr_nrm_beta_weights))
            return out, None
        x = self.lyr_nrm(query) if self.include_norm_add else query
        # the reference's self_attn_func / fast_self_attn_func
        out = self_attn(use_time_mask, is_training, self.num_heads, self.scaling, x, w, self.out_proj_weight, b,
                        self.out_proj_bias, mask, self.mask_additive, self.dropout, self.impl)
        if self.include_norm_add:
            out = dropout_add(out, query, self.dropout, is_training)
        return out, None
