"""Softmax cross-entropy with label smoothing (reference apex/contrib/xentropy/softmax_xentropy.py:4-28).

``SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing=0.0, padding_idx=0, half_to_float=False)``
returns per-row losses (rows whose label == padding_idx get 0 loss and 0 gradient).  GPU: the
single-pass gfx950 kernel in ``csrc/xentropy/xentropy.hip``; CPU: the same math in torch."""
import torch

from ... import _native


def _ext():
    return _native.require("xentropy_cuda").xentropy_cuda


def _torch_forward(logits, labels, smoothing, padding_idx):
    x = logits.float()
    lse = torch.logsumexp(x, dim=-1)
    log_prob = x.gather(1, labels.clamp(min=0).view(-1, 1)).squeeze(1) - lse
    losses = (lse - x.mean(-1)) * smoothing - log_prob * (1.0 - smoothing)
    losses = losses.masked_fill(labels == padding_idx, 0.0)
    return losses, lse


def _torch_backward(grad_loss, logits, lse, labels, smoothing, padding_idx):
    x = logits.float()
    classes = x.shape[-1]
    g = grad_loss.float().masked_fill(labels == padding_idx, 0.0).view(-1, 1)
    p = torch.exp(x - lse.view(-1, 1))
    onehot = torch.zeros_like(x).scatter_(1, labels.clamp(min=0).view(-1, 1), 1.0)
    return (g * (p - onehot * (1.0 - smoothing) - smoothing / classes)).to(logits.dtype)


class SoftmaxCrossEntropyLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing=0.0, padding_idx=0, half_to_float=False):
        if _native.use_native(logits):
            losses, lse = _ext().forward(logits, labels, float(smoothing), bool(half_to_float), int(padding_idx))
        else:
            losses, lse = _torch_forward(logits, labels, smoothing, padding_idx)
            if not half_to_float:
                losses = losses.to(logits.dtype)
        ctx.save_for_backward(logits, lse, labels)
        ctx.smoothing = float(smoothing)
        ctx.padding_idx = int(padding_idx)
        return losses

    @staticmethod
    def backward(ctx, grad_loss):
        logits, lse, labels = ctx.saved_tensors
        if _native.use_native(logits):
            grad = _ext().backward(grad_loss.contiguous(), logits, lse, labels, ctx.smoothing, ctx.padding_idx)
        else:
            grad = _torch_backward(grad_loss, logits, lse, labels, ctx.smoothing, ctx.padding_idx)
        return grad, None, None, None, None
