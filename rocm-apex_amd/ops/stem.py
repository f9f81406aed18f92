"""ResNet stem as ONE autograd node on native gfx950 kernels (``csrc/conv/stem.hip``):
``maxpool3x3/2(relu(bn(conv7x7/2(x))))`` for a training-mode BN.

Forward: the image is copied once into a zero-halo NHWC4 layout, the 7x7 convolution runs as an
MFMA implicit GEMM whose epilogue also accumulates the BN statistics, and one pass normalizes,
applies the ReLU and max-pools (1-byte window indices).  Backward: one pass gathers the pooled
gradient through the window indices, masks it with the recomputed ReLU and reduces the BN
backward sums; the weight-gradient kernel recomputes the BN input gradient from the same three
tensors as its operand prologue.  The full-resolution gradient never reaches HBM, and the
convolution's data gradient is never formed (the images need none).

Reference capability: the stem of the reference's ImageNet example
(``examples/imagenet/main_amp.py``: torchvision conv1 / bn1 / relu / maxpool) with the NHWC
batch norm of ``apex/contrib/groupbn``.  SyncBatchNorm (``bn_group > 1``) exchanges the
statistics and backward sums per step like the bottleneck node (``ops/bottleneck_bn.py``).

``APEX_AMD_NATIVE_STEM=0`` falls back to the module path (channel-padded library convolution,
fused NHWC BN + pool)."""
import os

import torch

from .. import _native
from . import bottleneck_bn as bb

_ENABLED = os.environ.get("APEX_AMD_NATIVE_STEM", "1") != "0"


def _ext():
    return _native.require("conv").conv


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, g, b, bn):
        y, part, xp = _ext().stem_fprop(x, w, bn.rm)
        m = float(y.size(0) * y.size(2) * y.size(3))
        sm, si, coef, inv_n = bb.finalize_part(part, m, bn)
        p, idx = _ext().stem_pool(y, coef)
        ctx.save_for_backward(xp, y, idx, w, g, sm, si, coef, inv_n)
        ctx.group = bn.group
        return p

    @staticmethod
    def backward(ctx, dp):
        xp, y, idx, w, g, sm, si, coef, inv_n = ctx.saved_tensors
        dp = dp.contiguous(memory_format=torch.channels_last)
        part = _ext().stem_reduce(dp, idx, y, coef, sm)
        m = float(y.size(0) * y.size(2) * y.size(3))
        cb, gg, gb = bb.bwd_from_part(part, m, sm, si, g, ctx.group, inv_n)
        dw = _ext().stem_wgrad(dp, idx, y, coef, cb.view(-1), xp, w)
        return None, dw, gg, gb, None


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def stem_supported(conv, bn, pool, x):
    """True when conv -> bn (+ReLU) -> pool is the ResNet stem shape the native node runs."""
    if not (_ENABLED and torch.is_tensor(x) and x.is_cuda and x.dim() == 4 and 1 <= x.size(1) <= 4
            and not x.requires_grad and _native.submodule("conv") is not None
            and not torch.is_autocast_enabled("cuda")):
        return False
    w = conv.weight
    if not (w.dtype in (torch.bfloat16, torch.float16) and tuple(w.shape) == (64, x.size(1), 7, 7)
            and _pair(conv.stride) == (2, 2) and _pair(conv.padding) == (3, 3) and _pair(conv.dilation) == (1, 1)
            and conv.groups == 1 and conv.bias is None):
        return False
    if not (bb._bn_ok(bn) and getattr(bn, "fuse_relu", False)):
        return False
    if not (_pair(pool.kernel_size) == (3, 3) and _pair(pool.stride or pool.kernel_size) == (2, 2)
            and _pair(pool.padding) == (1, 1) and _pair(getattr(pool, "dilation", 1)) == (1, 1)
            and not getattr(pool, "ceil_mode", False) and not getattr(pool, "return_indices", False)):
        return False
    # the module path would raise on a mismatch; an fp32 batch is taken only when amp O2 left its
    # cast to the model (models/resnet.py): the padding pass rounds it to w's dtype
    if x.dtype != w.dtype and not (x.dtype == torch.float32 and getattr(conv, "_amp_input_fp32_ok", False)):
        return False
    return not any(getattr(mod, attr, None) for mod in (conv, bn, pool)
                   for attr in ("_forward_hooks", "_forward_pre_hooks", "_backward_hooks", "_backward_pre_hooks"))


def stem_forward(conv, bn, pool, x):
    """The pooled stem output [N, 64, PH, PW] (channels_last) of ``x`` on the native node."""
    return _StemFn.apply(x, conv.weight, bn.weight, bn.bias, bb._BN(bn))
