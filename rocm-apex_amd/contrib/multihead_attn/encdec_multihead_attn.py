"""EncdecMultiheadAttn (reference apex/contrib/multihead_attn/encdec_multihead_attn.py:30-188):
query from the decoder, keys / values from the encoder output.  Parameter names match the
reference (``in_proj_weight_q``, ``in_proj_weight_kv`` [2E, E] interleaved per head as [k|v])."""
import math

import torch
from torch import nn
from torch.nn import Parameter

from ...normalization.fused_layer_norm import FusedLayerNorm
from ._core import dropout_add, encdec_attn


class EncdecMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False, impl="fast"):
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
        self.in_proj_weight_q = Parameter(torch.empty(embed_dim, embed_dim))
        self.in_proj_weight_kv = Parameter(torch.empty(2 * embed_dim, embed_dim))
        self.out_proj_weight = Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            self.in_proj_bias_q = Parameter(torch.empty(embed_dim))
            self.in_proj_bias_kv = Parameter(torch.empty(2 * embed_dim))
            self.out_proj_bias = Parameter(torch.empty(embed_dim))
        else:
            self.register_parameter("in_proj_bias_q", None)
            self.register_parameter("in_proj_bias_kv", None)
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
        nn.init.xavier_uniform_(self.in_proj_weight_q)
        # [2E, E] initialised like an [E, E] matrix (reference :84-87)
        nn.init.xavier_uniform_(self.in_proj_weight_kv, gain=math.sqrt(1.5))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            nn.init.constant_(self.in_proj_bias_q, 0.0)
            nn.init.constant_(self.in_proj_bias_kv, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)
        if self.include_norm_add:
            if self.impl == "fast":
                nn.init.ones_(self.lyr_nrm_gamma_weights)
                nn.init.zeros_(self.lyr_nrm_beta_weights)
            else:
                self.lyr_nrm.reset_parameters()

    def forward(self, query, key, value, key_padding_mask=None, need_weights=False, attn_mask=None,
                is_training=True):
        """query [sq, batch, embed]; key [sk, batch, embed] (value ignored: kv share one projection)."""
        if key_padding_mask is not None:
            assert attn_mask is None, "ERROR attn_mask and key_padding_mask should not be both defined!"
        mask = key_padding_mask if key_padding_mask is not None else attn_mask
        use_time_mask = attn_mask is not None
        weights = (self.in_proj_weight_q, self.in_proj_weight_kv, self.out_proj_weight, self.in_proj_bias_q,
                   self.in_proj_bias_kv, self.out_proj_bias)
        if self.include_norm_add and self.impl == "fast":
            # the reference's fast_encdec_attn_norm_add_func
            out = encdec_attn(use_time_mask, is_training, self.num_heads, self.scaling, query, key, *weights, mask,
                              self.dropout, "fast", norm=(self.lyr_nrm_gamma_weights, self.lyr_nrm_beta_weights))
            return out, None
        x = self.lyr_nrm(query) if self.include_norm_add else query
        # the reference's encdec_attn_func / fast_encdec_attn_func
        out = encdec_attn(use_time_mask, is_training, self.num_heads, self.scaling, x, key, *weights, mask,
                          self.dropout, self.impl)
        if self.include_norm_add:
            out = dropout_add(out, query, self.dropout, is_training)
        return out, None
