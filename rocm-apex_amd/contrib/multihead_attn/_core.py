"""Shared attention core of SelfMultiheadAttn / EncdecMultiheadAttn.

``impl="fast"``: projections are plain library GEMMs (hipBLASLt through ``F.linear``); the
attention itself is ONE fused flash kernel launch per direction reading Q/K/V straight out of the
interleaved projection output (strided views, no permute copies) and writing the context in the
``[seq, batch, embed]`` layout the output projection consumes.  The reference's fast path
(apex/contrib/csrc/multihead_attn/self_multihead_attn_cuda.cu) instead runs two strided-batched
GEMMs around a materialised [b*h, sq, sk] softmax + dropout-mask tensor.

``impl="default"``: explicit torch math (matmul / softmax / dropout), the reference's python
path (apex/contrib/multihead_attn/self_multihead_attn_func.py), kept as an independent check.

Masks (reference semantics): ``key_padding_mask`` [batch, sk] (bool/byte: 1 = padded, or an
additive float mask when ``mask_additive``), ``attn_mask`` ("time mask") [sq, sk] bool, 1 = hidden.
"""
import torch
import torch.nn.functional as F

from ...ops.attention import flash_attn_func


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
