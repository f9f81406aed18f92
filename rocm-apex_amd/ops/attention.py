"""Fused attention entry point (``apex.ops.attention.flash_attn_func``).

GPU tensors with head dim 32 / 64 / 128 in fp16 / bf16 run the gfx950 flash kernels
(``csrc/attn/flash_attn.hip``: in-register online softmax, P fed to P·V from registers, no
sq x sk tensor in HBM); everything else runs the torch reference math below, which uses the
SAME counter-based dropout hash so CPU and GPU results agree mask-for-mask.

Layouts: padded ``[batch, seq, heads, d]`` or varlen ``[total, heads, d]`` with ``cu_seqlens``
(any strides with d contiguous — e.g. views into an interleaved QKV projection output).
``bias`` is an additive fp32 mask broadcastable to ``[batch, heads, sq, sk]``.
Causal masking is top-left aligned (key j visible to query i iff j <= i), as in the
reference's time mask (apex/contrib/multihead_attn/self_multihead_attn_func.py:58-63).
"""
import math

import torch

from .. import _native
from . import dropout_rng

_M32 = 0xFFFFFFFF


def _mix32(x):
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def seed_mix(seed, offset):
    seed, offset = int(seed) & ((1 << 64) - 1), int(offset) & ((1 << 64) - 1)
    x = (seed & _M32) ^ (((seed >> 32) * 0x27D4EB2D) & _M32) ^ (((offset & _M32) * 0x165667B1) & _M32) ^ \
        ((((offset >> 32) & _M32) * 0xD3A2646C) & _M32)
    x &= _M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & _M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def dropout_keep_mask(seed, offset, bh, sq, sk, p, device="cpu"):
    """Keep mask [len(bh), sq, sk] of the kernels' dropout for flat (batch*heads) indices ``bh``."""
    sm = seed_mix(seed, offset)
    bh = torch.as_tensor(bh, dtype=torch.int64, device=device).view(-1, 1, 1)
    q = torch.arange(sq, dtype=torch.int64, device=device).view(1, -1, 1)
    k = torch.arange(sk, dtype=torch.int64, device=device).view(1, 1, -1)
    a = _mix32(sm ^ ((bh * 0x9E3779B9) & _M32))
    row = _mix32(a ^ ((q * 0x85EBCA6B) & _M32))
    # one hash per key pair (k >> 1): the even key tests the low 16 bits, the odd key the high
    h = _mix32(row ^ (((k >> 1) * 0xC2B2AE35) & _M32))
    bits = torch.where((k & 1) == 1, h >> 16, h & 0xFFFF)
    return bits >= min(int(p * 65536.0), 65536)


def dropout_keep_scale(p):
    """1 / the kernels' exact keep rate: (65536 - t16) / 65536 of the 16-bit tests survive
    (t16 = floor(p * 65536)), so the unbiased scale is 65536 / (65536 - t16), not 1 / (1 - p)."""
    t16 = min(int(p * 65536.0), 65536)
    return 65536.0 / (65536 - t16) if t16 < 65536 else 0.0


def _native_ok(q, k, v, bias):
    if not (q.is_cuda and _native.use_native(q)):
        return False
    if q.dtype not in (torch.float16, torch.bfloat16) or q.size(-1) not in (32, 64, 128):
        return False
    for t in (q, k, v):
        if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:-1]) or t.data_ptr() % 16:
            return False
    return True


def _ref_attention(q, k, v, scale, causal, bias, p, seed, offset, cu_q, cu_k):
    """fp32 torch math with the kernels' semantics; returns (out, lse[h, rows])."""
    if cu_q is not None:
        outs, lses = [], []
        cq, ck = cu_q.tolist(), cu_k.tolist()
        for bi in range(len(cq) - 1):
            qs, ks = q[cq[bi]:cq[bi + 1]].unsqueeze(0), k[ck[bi]:ck[bi + 1]].unsqueeze(0)
            vs = v[ck[bi]:ck[bi + 1]].unsqueeze(0)
            bb = None if bias is None else bias[min(bi, bias.size(0) - 1):min(bi, bias.size(0) - 1) + 1]
            o, l = _ref_padded(qs, ks, vs, scale, causal, bb, p, seed, offset, bi)
            outs.append(o[0])
            lses.append(l)
        return torch.cat(outs, 0), torch.cat(lses, 1)
    return _ref_padded(q, k, v, scale, causal, bias, p, seed, offset, None)


def _ref_padded(q, k, v, scale, causal, bias, p, seed, offset, batch_index):
    B, Sq, H, D = q.shape
    Sk, Hk = k.size(1), k.size(2)
    rep = H // Hk
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, 1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if bias is not None:
        s = s + bias.float()
    if causal:
        mask = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    m = s.amax(-1, keepdim=True)
    m = torch.where(torch.isinf(m), torch.zeros_like(m), m)
    e = torch.exp(s - m)
    l = e.sum(-1, keepdim=True)
    probs = torch.where(l > 0, e / l, torch.zeros_like(e))
    lse = torch.where(l > 0, (m + torch.log(l)), torch.full_like(l, float("inf"))).squeeze(-1)  # [B, H, Sq]
    if p > 0:
        b0 = 0 if batch_index is None else batch_index
        bh = (torch.arange(B).view(B, 1) + b0) * H + torch.arange(H).view(1, H)
        keep = dropout_keep_mask(seed, offset, bh.view(-1), Sq, Sk, p, q.device).view(B, H, Sq, Sk)
        probs = probs * keep * dropout_keep_scale(p)
    out = torch.matmul(probs, vf).transpose(1, 2).to(q.dtype)
    return out, lse.permute(1, 0, 2).reshape(H, B * Sq)


class FlashAttnFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, bias, p, seed, offset, cu_q, cu_k, max_q, max_k):
        native = _native_ok(q, k, v, bias)
        if native:
            C = _native.require("flash attention")
            b = None if bias is None else bias.float()
            if b is not None:
                while b.dim() < 4:
                    b = b.unsqueeze(0)
            step = dropout_rng.snapshot(q.device) if p > 0 else None
            out, lse = C.attn.fwd(q, k, v, cu_q, cu_k, max_q, max_k, scale, causal, b, p, seed, offset,
                                  rng_step=step)
            ctx.save_for_backward(q, k, v, out, lse, b, cu_q, cu_k)
            ctx.rng_step = step
        else:
            with torch.enable_grad():
                qq, kk, vv = (t.detach().requires_grad_(t.requires_grad) for t in (q, k, v))
                off = dropout_rng.effective_offset(offset, q.device) if p > 0 else offset
                out_g, lse = _ref_attention(qq, kk, vv, scale, causal, bias, p, seed, off, cu_q, cu_k)
            ctx.ref_graph = (qq, kk, vv, out_g)
            out = out_g.detach()
        ctx.native = native
        ctx.meta = (scale, causal, p, seed, offset, max_q, max_k)
        return out

    @staticmethod
    def backward(ctx, dout):
        scale, causal, p, seed, offset, max_q, max_k = ctx.meta
        if ctx.native:
            q, k, v, out, lse, b, cu_q, cu_k = ctx.saved_tensors
            C = _native.require("flash attention backward")
            dq, dk, dv = C.attn.bwd(dout, q, k, v, out, lse, cu_q, cu_k, max_q, max_k, scale, causal, b, p, seed,
                                    offset, rng_step=ctx.rng_step)
        else:
            qq, kk, vv, out_g = ctx.ref_graph
            need = [t for t in (qq, kk, vv) if t.requires_grad]
            grads = torch.autograd.grad(out_g, need, dout, allow_unused=True) if need else []
            it = iter(grads)
            dq, dk, dv = (next(it) if t.requires_grad else None for t in (qq, kk, vv))
        return dq, dk, dv, None, None, None, None, None, None, None, None, None, None


_offset_counter = [0]


def next_dropout_seed(device=None):
    """(seed, offset) pair for one dropout call: seed from torch's generator, offset counter."""
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,), generator=None).item())
    _offset_counter[0] += 1
    return seed, _offset_counter[0]


def flash_attn_func(q, k, v, dropout_p=0.0, softmax_scale=None, causal=False, bias=None, cu_seqlens_q=None,
                    cu_seqlens_k=None, max_seqlen_q=None, max_seqlen_k=None, seed=None, offset=None):
    """softmax(scale * q k^T + bias [causal]) (dropout) v over heads; see module docstring."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.size(-1))
    if dropout_p > 0 and seed is None:
        seed, offset = next_dropout_seed()
    seed = 0 if seed is None else int(seed)
    offset = 0 if offset is None else int(offset)
    if cu_seqlens_q is not None:
        if max_seqlen_q is None:
            max_seqlen_q = int((cu_seqlens_q[1:] - cu_seqlens_q[:-1]).max())
        if max_seqlen_k is None:
            max_seqlen_k = int((cu_seqlens_k[1:] - cu_seqlens_k[:-1]).max())
    else:
        max_seqlen_q, max_seqlen_k = q.size(1), k.size(1)
    return FlashAttnFunc.apply(q, k, v, float(scale), bool(causal), bias, float(dropout_p), seed, offset,
                               cu_seqlens_q, cu_seqlens_k, int(max_seqlen_q), int(max_seqlen_k))


class _PackedQKVSelfAttention(torch.autograd.Function):
    """Self-attention from a fused QKV projection in Megatron layout ``[s, b, heads, 3*d]`` to the
    context ``[s, b, heads*d]``.  Q / K / V are strided views of the projection, the forward
    kernel writes the context directly in ``[s, b]`` order and the backward kernel writes dQ / dK /
    dV into one d(QKV) buffer — autograd never sees the three slices, so there is no per-slice
    zero-filled gradient, copy and sum, and no transpose copy of the context or its gradient."""

    @staticmethod
    def forward(ctx, mixed, scale, causal, bias, p, seed, offset):
        C = _native.require("flash attention")
        s, b, nh, three_d = mixed.shape
        d = three_d // 3
        q, k, v = (mixed[..., i * d:(i + 1) * d].permute(1, 0, 2, 3) for i in range(3))
        out = torch.empty(s, b, nh, d, device=mixed.device, dtype=mixed.dtype)
        bias4 = None if bias is None else bias.float()
        if bias4 is not None:
            while bias4.dim() < 4:
                bias4 = bias4.unsqueeze(0)
        step = dropout_rng.snapshot(mixed.device) if p > 0 else None
        _, lse = C.attn.fwd(q, k, v, None, None, 0, 0, scale, causal, bias4, p, seed, offset, out.permute(1, 0, 2, 3),
                            rng_step=step)
        ctx.save_for_backward(mixed, out, lse, bias4)
        ctx.meta = (scale, causal, p, seed, offset)
        ctx.rng_step = step
        return out.view(s, b, nh * d)

    @staticmethod
    def backward(ctx, dout):
        C = _native.require("flash attention backward")
        mixed, out, lse, bias4 = ctx.saved_tensors
        scale, causal, p, seed, offset = ctx.meta
        s, b, nh, three_d = mixed.shape
        d = three_d // 3
        q, k, v = (mixed[..., i * d:(i + 1) * d].permute(1, 0, 2, 3) for i in range(3))
        dmixed = torch.empty_like(mixed)
        dq, dk, dv = (dmixed[..., i * d:(i + 1) * d].permute(1, 0, 2, 3) for i in range(3))
        g = dout.contiguous().view(s, b, nh, d).permute(1, 0, 2, 3)
        C.attn.bwd(g, q, k, v, out.permute(1, 0, 2, 3), lse, None, None, 0, 0, scale, causal, bias4, p, seed, offset,
                   dq, dk, dv, rng_step=ctx.rng_step)
        return dmixed, None, None, None, None, None, None


def packed_qkv_self_attention(mixed, scale, causal=False, bias=None, dropout_p=0.0, seed=0, offset=0):
    """``[s, b, heads, 3*d]`` fused-QKV projection -> ``[s, b, heads*d]`` attention context
    (Megatron self-attention layout; see :class:`_PackedQKVSelfAttention`).  Non-native inputs
    take :func:`flash_attn_func` on the q / k / v views."""
    s, b, nh, three_d = mixed.shape
    d = three_d // 3
    q, k, v = (mixed[..., i * d:(i + 1) * d].permute(1, 0, 2, 3) for i in range(3))
    if _native_ok(q, k, v, bias) and mixed.is_contiguous():
        return _PackedQKVSelfAttention.apply(mixed, float(scale), bool(causal), bias, float(dropout_p), int(seed),
                                             int(offset))
    ctx = flash_attn_func(q, k, v, dropout_p=dropout_p, softmax_scale=scale, causal=causal, bias=bias, seed=seed,
                          offset=offset)
    return ctx.transpose(0, 1).reshape(s, b, nh * d)
