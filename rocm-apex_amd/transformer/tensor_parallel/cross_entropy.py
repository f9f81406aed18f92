"""Cross entropy over a vocabulary sharded across the tensor-parallel group
(reference apex/transformer/tensor_parallel/cross_entropy.py:23-103).

Collectives: the reference issues three all-reduces per call (MAX of the logits, SUM of the
target logit, SUM of exp).  Here the two SUM reductions are packed into ONE all-reduce of a
[2, tokens] fp32 tensor, so the op costs two latency-bound RCCL calls instead of three.
The softmax is kept in fp32 for the backward (same as the reference), label smoothing is
supported (Megatron-LM semantics)."""
import torch

from ..parallel_state import get_tensor_model_parallel_group, get_tensor_model_parallel_rank, \
    get_tensor_model_parallel_world_size
from .utils import VocabUtility


class _VocabParallelCrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, vocab_parallel_logits, target, label_smoothing=0.0):
        logits = vocab_parallel_logits.float()
        group = get_tensor_model_parallel_group()
        world = get_tensor_model_parallel_world_size()
        logits_max = torch.max(logits, dim=-1)[0]
        if world > 1:
            torch.distributed.all_reduce(logits_max, op=torch.distributed.ReduceOp.MAX, group=group)
        logits = logits - logits_max.unsqueeze(dim=-1)

        partition_vocab_size = logits.size()[-1]
        vocab_start, vocab_end = VocabUtility.vocab_range_from_per_partition_vocab_size(
            partition_vocab_size, get_tensor_model_parallel_rank(), world)
        target_mask = (target < vocab_start) | (target >= vocab_end)
        masked_target = target.clone() - vocab_start
        masked_target[target_mask] = 0

        logits_2d = logits.view(-1, partition_vocab_size)
        masked_target_1d = masked_target.view(-1)
        arange_1d = torch.arange(0, logits_2d.size()[0], device=logits_2d.device)
        predicted = logits_2d[arange_1d, masked_target_1d].clone().view_as(target)
        predicted[target_mask] = 0.0

        exp_logits = torch.exp(logits)
        sum_exp = exp_logits.sum(dim=-1)
        packed = torch.stack([predicted.float(), sum_exp.float()])
        if world > 1:
            torch.distributed.all_reduce(packed, op=torch.distributed.ReduceOp.SUM, group=group)
        predicted, sum_exp = packed[0], packed[1]

        loss = torch.log(sum_exp) - predicted
        exp_logits.div_(sum_exp.unsqueeze(dim=-1))
        vocab_size = partition_vocab_size * world
        if label_smoothing > 0:
            # loss = (1 - s) * nll + s * mean_over_vocab(-log p)
            log_probs = torch.log(exp_logits.clamp_min(1e-30))
            sum_log_probs = log_probs.sum(dim=-1)
            if world > 1:
                torch.distributed.all_reduce(sum_log_probs, group=group)
            smoothing = label_smoothing * vocab_size / (vocab_size - 1)
            loss = (1.0 - smoothing) * loss - smoothing * sum_log_probs / vocab_size
        ctx.label_smoothing = label_smoothing
        ctx.vocab_size = vocab_size
        ctx.save_for_backward(exp_logits, target_mask, masked_target_1d)
        return loss

    @staticmethod
    def backward(ctx, grad_output):
        softmax, target_mask, masked_target_1d = ctx.saved_tensors
        grad_input = softmax
        partition_vocab_size = softmax.size()[-1]
        grad_2d = grad_input.view(-1, partition_vocab_size)
        arange_1d = torch.arange(0, grad_2d.size()[0], device=grad_2d.device)
        update = 1.0 - target_mask.view(-1).float()
        if ctx.label_smoothing > 0:
            smoothing = ctx.label_smoothing * ctx.vocab_size / (ctx.vocab_size - 1)
            grad_2d[arange_1d, masked_target_1d] -= (1.0 - smoothing) * update
            grad_2d -= smoothing / ctx.vocab_size
        else:
            grad_2d[arange_1d, masked_target_1d] -= update
        grad_input.mul_(grad_output.unsqueeze(dim=-1))
        return grad_input, None, None


class _FusedCrossEntropy(torch.autograd.Function):
    """Unsharded vocabulary (TP world 1) on a GPU: the gfx950 softmax cross-entropy kernel of
    apex.contrib.xentropy run straight on the bf16 / fp16 logits (fp32 math inside) — one read of
    the [tokens, vocab] logits forward, one read + one write backward, instead of an fp32 copy, a
    materialised fp32 softmax and five elementwise / reduction passes.  Megatron's label
    smoothing s maps onto the kernel's as s * V / (V - 1) (same loss, same gradient)."""

    @staticmethod
    def forward(ctx, logits, target, label_smoothing):
        from ... import _native

        ext = _native.require("xentropy_cuda").xentropy_cuda
        v = logits.size(-1)
        x2 = logits.reshape(-1, v)
        t1 = target.reshape(-1)
        s = label_smoothing * v / (v - 1) if label_smoothing > 0 else 0.0
        losses, lse = ext.forward(x2, t1, float(s), True, None)
        ctx.save_for_backward(x2, lse, t1)
        ctx.smoothing = s
        ctx.shape = logits.shape
        return losses.view(target.shape)

    @staticmethod
    def backward(ctx, grad_output):
        from ... import _native

        x2, lse, t1 = ctx.saved_tensors
        grad = _native.require("xentropy_cuda").xentropy_cuda.backward(
            grad_output.reshape(-1).float().contiguous(), x2, lse, t1, ctx.smoothing, None)
        return grad.view(ctx.shape), None, None


def _fused_ok(logits):
    from ... import _native

    return (get_tensor_model_parallel_world_size() == 1 and logits.is_cuda and _native.use_native(logits)
            and _native.submodule("xentropy_cuda") is not None
            and logits.dtype in (torch.float16, torch.bfloat16, torch.float32))


def vocab_parallel_cross_entropy(vocab_parallel_logits, target, label_smoothing=0.0):
    """Per-token loss for logits sharded along the vocabulary over the TP group (fp32 math;
    low-precision logits are upcast inside, never materialised in fp32 on the fused path)."""
    if _fused_ok(vocab_parallel_logits):
        return _FusedCrossEntropy.apply(vocab_parallel_logits, target, label_smoothing)
    return _VocabParallelCrossEntropy.apply(vocab_parallel_logits, target, label_smoothing)
