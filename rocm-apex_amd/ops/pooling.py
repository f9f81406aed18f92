"""Channels-last max pooling (``csrc/pool/maxpool_nhwc.hip``): 1-byte window indices instead of
PyTorch's int64 ones and a gather-form backward.  ``MaxPool2dNHWC`` is a drop-in for
``nn.MaxPool2d`` that takes the native path for channels_last GPU inputs with C % 8 == 0 and
the torch op otherwise."""
import torch
import torch.nn.functional as F

from .. import _native


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        lib = _native.require("maxpool_nhwc").maxpool_nhwc
        y, idx = lib.forward(x, list(k), list(s), list(p))
        ctx.save_for_backward(idx)
        ctx.meta = (k, s, p, x.shape, x.dtype, x.device)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        k, s, p, shape, dtype, dev = ctx.meta
        # shape / layout carrier only: allocate channels_last directly (a .to(memory_format=) here
        # was a 411 MB copy per step on the ResNet-50 stem)
        x_like = torch.empty(shape, dtype=dtype, device=dev, memory_format=torch.channels_last)
        dx = _native.require("maxpool_nhwc").maxpool_nhwc.backward(dy, idx, x_like, list(k), list(s), list(p))
        return dx, None, None, None


def max_pool2d_nhwc(x, kernel_size, stride=None, padding=0):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and x.size(1) % 8 == 0
            and x.dtype in (torch.float16, torch.bfloat16, torch.float32) and _native.submodule("maxpool_nhwc")
            is not None):
        return _MaxPoolNHWC.apply(x, k, s, p)
    return F.max_pool2d(x, k, s, p)


class MaxPool2dNHWC(torch.nn.MaxPool2d):
    def forward(self, x):
        if self.dilation not in (1, (1, 1)) or self.ceil_mode or self.return_indices:
            return super().forward(x)
        return max_pool2d_nhwc(x, self.kernel_size, self.stride, self.padding)
