"""Shared attention core of SelfMultiheadAttn / EncdecMultiheadAttn.

``impl="fast"``: projections are plain library GEMMs (hipBLASLt through ``F.linear``); the
attention itself is ONE fused flash kernel launch per direction reading Q/K/V straight out of the
interleaved projection output (strided views, no permute copies) and writing the context in the
``[seq, batch, embed]`` layout the output projection consumes.  Self-attention hands the
projection output to the packed-QKV kernel pair as ``[seq, batch, heads, 3*head_dim]``: the
backward writes dQ / dK / dV into ONE gradient buffer of the projection, so autograd never forms
the three zero-filled slice gradients and their sum (host launches and device passes per layer).  The reference's fast path
(apex/contrib/csrc/multihead_attn/self_multihead_attn_cuda.cu) instead runs two strided-batched
GEMMs around a materialised [b*h, sq, sk] softmax + dropout-mask tensor.

``impl="default"``: explicit torch math (matmul / softmax / dropout), the reference's python
path (apex/contrib/multihead_attn/self_multihead_attn_func.py), kept as an independent check.

Masks (reference semantics): ``key_padding_mask`` [batch, sk] (bool/byte: 1 = padded, or an
additive float mask when ``mask_additive``), ``attn_mask`` ("time mask") [sq, sk] bool, 1 = hidden.
"""
import torch
import torch.nn.functional as F

from ...ops.attention import flash_attn_func, next_dropout_seed, packed_qkv_self_attention


def mask_to_bias(key_padding_mask, attn_mask, mask_additive, batch, sq, sk, device):
    """Reference masks -> additive fp32 bias broadcastable to [b, h, sq, sk] (None if no mask)."""
    if key_padding_mask is not None:
        m = key_padding_mask
        if mask_additive:
            bias = m.to(device=device, dtype=torch.float32)
        else:
            bias = torch.zeros(m.shape, dtype=torch.float32, device=device).masked_fill_(m.to(device).bool(),
                                                                                       float("-inf"))
        return bias.view(batch, 1, 1, sk)
    if attn_mask is not None:
        assert attn_mask.dim() == 2, "Timing mask is not 2D!"
        bias = torch.zeros(attn_mask.shape, dtype=torch.float32, device=device).masked_fill_(
            attn_mask.to(device).bool(), float("-inf"))
        return bias.view(1, 1, sq, sk)
    return None


def attention(q4, k4, v4, bias, scale, dropout, is_training, impl):
    """q4 [b, sq, h, d], k4/v4 [b, sk, h, d] (strided views) -> context [sq, b, h*d] contiguous."""
    b, sq, h, d = q4.shape
    p = dropout if is_training else 0.0
    if impl == "fast":
        ctx = flash_attn_func(q4, k4, v4, dropout_p=p, softmax_scale=scale, bias=bias)
        return ctx.transpose(0, 1).reshape(sq, b, h * d)
    # default: explicit torch math on [b*h, s, d]
    qf = q4.permute(0, 2, 1, 3).reshape(b * h, sq, d)
    kf = k4.permute(0, 2, 1, 3).reshape(b * h, k4.size(1), d)
    vf = v4.permute(0, 2, 1, 3).reshape(b * h, k4.size(1), d)
    s = torch.bmm(qf, kf.transpose(1, 2)) * scale
    if bias is not None:
        s = (s.view(b, h, sq, -1) + bias.to(s.dtype)).view(b * h, sq, -1)
    probs = F.softmax(s.float(), dim=-1).to(q4.dtype)
    if p > 0:
        probs = F.dropout(probs, p=p, training=True)
    ctx = torch.bmm(probs, vf)  # [b*h, sq, d]
    return ctx.view(b, h, sq, d).permute(2, 0, 1, 3).reshape(sq, b, h * d)


def split_heads_interleaved(lin, seq, batch, heads, parts):
    """[seq, batch, heads*parts*d] projection output -> ``parts`` [batch, seq, heads, d] views
    (the reference's ``view(seq, batch*heads, parts, d)`` interleave)."""
    d = lin.size(-1) // (heads * parts)
    v = lin.view(seq, batch, heads, parts, d)
    return [v[:, :, :, i].permute(1, 0, 2, 3) for i in range(parts)]


def dropout_add(x, residual, p, is_training):
    if is_training and p > 0:
        x = F.dropout(x, p=p, training=True)
    return x + residual


def _masks(use_time_mask, mask):
    """The reference's single ``mask`` argument -> (key_padding_mask, attn_mask)."""
    return (None, mask) if use_time_mask else (mask, None)


def self_attn(use_time_mask, is_training, heads, scale, inputs, input_weights, output_weights, input_biases,
              output_biases, mask, mask_additive, dropout_prob, impl, norm=None):
    """Self attention as the reference's ``*self_attn*_func`` API: inputs [seq, batch, E],
    input_weights [3E, E] interleaved per head as [q|k|v]; ``norm`` = (gamma, beta) runs the
    fused LayerNorm on the input first and adds the dropped-out result to ``inputs`` (norm_add)."""
    from ...normalization.fused_layer_norm import fused_layer_norm_affine

    seq, batch, e = inputs.shape
    x = inputs if norm is None else fused_layer_norm_affine(inputs, norm[0], norm[1], (e,), 1e-5)
    lin = F.linear(x, input_weights, input_biases)
    kpm, am = _masks(use_time_mask, mask)
    bias = mask_to_bias(kpm, am, mask_additive, batch, seq, seq, inputs.device)
    if impl == "fast":
        p = dropout_prob if is_training else 0.0
        seed, offset = next_dropout_seed() if p > 0 else (0, 0)
        ctx = packed_qkv_self_attention(lin.view(seq, batch, heads, -1), scale, False, bias, p, seed, offset)
    else:
        q4, k4, v4 = split_heads_interleaved(lin, seq, batch, heads, 3)
        ctx = attention(q4, k4, v4, bias, scale, dropout_prob, is_training, impl)
    out = F.linear(ctx, output_weights, output_biases)
    return out if norm is None else dropout_add(out, inputs, dropout_prob, is_training)


def encdec_attn(use_time_mask, is_training, heads, scale, inputs_q, inputs_kv, input_weights_q, input_weights_kv,
                output_weights, input_biases_q, input_biases_kv, output_biases, mask, dropout_prob, impl,
                norm=None):
    """Encoder-decoder attention as the reference's ``*encdec_attn*_func`` API: queries from
    ``inputs_q`` [sq, batch, E], keys / values from ``inputs_kv`` [sk, batch, E] through one [2E, E]
    projection interleaved per head as [k|v]."""
    from ...normalization.fused_layer_norm import fused_layer_norm_affine

    sq, batch, e = inputs_q.shape
    sk = inputs_kv.size(0)
    x = inputs_q if norm is None else fused_layer_norm_affine(inputs_q, norm[0], norm[1], (e,), 1e-5)
    lq = F.linear(x, input_weights_q, input_biases_q)
    lkv = F.linear(inputs_kv, input_weights_kv, input_biases_kv)
    (q4,) = split_heads_interleaved(lq, sq, batch, heads, 1)
    k4, v4 = split_heads_interleaved(lkv, sk, batch, heads, 2)
    kpm, am = _masks(use_time_mask, mask)
    bias = mask_to_bias(kpm, am, False, batch, sq, sk, inputs_q.device)
    ctx = attention(q4, k4, v4, bias, scale, dropout_prob, is_training, impl)
    out = F.linear(ctx, output_weights, output_biases)
    return out if norm is None else dropout_add(out, inputs_q, dropout_prob, is_training)


class FuncNamespace:
    """Reference modules expose ``XxxFunc`` autograd classes next to ``xxx_func = XxxFunc.apply``;
    here the functions are compositions of autograd-capable ops (the flash-attention Function,
    fused LayerNorm, linear), so the class only carries ``apply``."""

    def __init_subclass__(cls, fn=None, **kw):
        super().__init_subclass__(**kw)
        cls.apply = staticmethod(fn)
