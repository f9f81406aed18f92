"""Fused multi-head attention for packed variable-length batches (reference
apex/contrib/fmha/fmha.py:33-74).

``qkv`` is ``[total_tokens, 3, heads, d]`` with ``cu_seqlens`` [batch + 1] int32 prefix sums.
The reference is sm80-only (head dim 64, seq <= 512, fp16); here any seq length, head dim
32 / 64 / 128 and fp16 / bf16 run the gfx950 flash kernels (``_C.fmhalib``), and CPU tensors the
torch reference math of :mod:`apex.ops.attention`."""
import torch

from ... import _native
from ...ops import attention as _attn


class FMHAFun(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cu_seqlens, p_dropout, max_s, is_training, zero_tensors=False):
        p = p_dropout if is_training else 0.0
        seed, offset = _attn.next_dropout_seed() if p > 0 else (0, 0)
        native = qkv.is_cuda and qkv.size(-1) in (32, 64, 128) and qkv.dtype in (torch.float16, torch.bfloat16)
        if native:
            lib = _native.require("fmha").fmhalib
            context, lse, meta = lib.fwd(qkv, cu_seqlens.int(), p, int(max_s), bool(is_training), seed, offset)
            ctx.save_for_backward(qkv, context, lse, meta, cu_seqlens)
        else:
            q, k, v = qkv.unbind(1)
            context = _attn.flash_attn_func(q, k, v, dropout_p=p, cu_seqlens_q=cu_seqlens, cu_seqlens_k=cu_seqlens,
                                            max_seqlen_q=max_s, max_seqlen_k=max_s, seed=seed, offset=offset)
            ctx.save_for_backward(qkv, cu_seqlens)
        ctx.native = native
        ctx.p = p
        ctx.max_s = max_s
        ctx.seed_offset = (seed, offset)
        return context

    @staticmethod
    def backward(ctx, dout):
        if ctx.native:
            qkv, context, lse, meta, cu = ctx.saved_tensors
            (dqkv,) = _native.require("fmha").fmhalib.bwd(dout.contiguous(), qkv, context, lse, meta, cu.int(), ctx.p,
                                                         int(ctx.max_s))
        else:
            qkv, cu = ctx.saved_tensors
            with torch.enable_grad():
                x = qkv.detach().requires_grad_(True)
                q, k, v = x.unbind(1)
                seed, offset = ctx.seed_offset
                out = _attn.flash_attn_func(q, k, v, dropout_p=ctx.p, cu_seqlens_q=cu, cu_seqlens_k=cu,
                                            max_seqlen_q=ctx.max_s, max_seqlen_k=ctx.max_s, seed=seed, offset=offset)
                (dqkv,) = torch.autograd.grad(out, [x], dout)
        return dqkv, None, None, None, None, None


class FMHA(torch.nn.Module):
    def __init__(self, config):
        super().__init__()
        self.p_dropout = config.attention_probs_dropout_prob
        self.h = config.num_attention_heads
        self.hidden_size = config.hidden_size
        self.d = self.hidden_size // self.h
        assert self.d * self.h == self.hidden_size, "Invalid hidden size/num_heads"

    def forward(self, qkv, cu_seqlens, max_s, is_training=True, zero_tensors=False):
        ctx = FMHAFun.apply(qkv.view(-1, 3, self.h, self.d), cu_seqlens, self.p_dropout, max_s, is_training,
                            zero_tensors)
        return ctx.view(-1, self.hidden_size)

