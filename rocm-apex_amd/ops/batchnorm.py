"""Batch-norm statistics / apply primitives used by SyncBatchNorm and the fused NHWC BN
(reference csrc/syncbn.cpp:8-109).

GPU tensors run the gfx950 Welford kernels (``_C.syncbn``, csrc/syncbn/welford.hip); CPU tensors
use the torch implementations below, which are also the numerics oracle in tests.
Layouts: ``channel_last=False`` -> [N, C, *]; ``channel_last=True`` -> [..., C] (the channel is
the LAST logical dim; torch channels_last activations are passed in as a permuted NHWC view).

Fused ReLU: ``batchnorm_forward(..., z, fuse_relu)`` computes relu(bn(x) + z); the backward
helpers accept the same (z, bias, fuse_relu) and mask the gradient by the recomputed output."""
import torch

from .. import _native


def _syncbn():
    return _native.require("syncbn").syncbn


def _reduce_dims(x, channel_last):
    if channel_last:
        return tuple(range(x.dim() - 1))
    return (0,) + tuple(range(2, x.dim()))


def _bshape(x, channel_last):
    if channel_last:
        return (1,) * (x.dim() - 1) + (-1,)
    return (1, -1) + (1,) * (x.dim() - 2)


def _c(t):
    return None if t is None else t.contiguous()


def welford_mean_var(x, channel_last=False):
    """Per-channel mean and biased variance (fp32 outputs)."""
    if _native.use_native(x):
        m = _syncbn()
        x = x.contiguous()
        return tuple(m.welford_mean_var_c_last(x) if channel_last else m.welford_mean_var(x))
    xf = x.float()
    dims = _reduce_dims(xf, channel_last)
    mean = xf.mean(dim=dims)
    var = xf.var(dim=dims, unbiased=False)
    return mean, var


def welford_parallel(mean_all, var_all, count_all, eps):
    """Merge per-rank (mean, biased var, count) -> (mean, unbiased var, inv_std)."""
    if _native.use_native(mean_all):
        return tuple(_syncbn().welford_parallel(mean_all, var_all, count_all.to(torch.int32), float(eps)))
    cnt = count_all.double().view(-1, 1)
    n = cnt.sum(0)
    mean = (mean_all.double() * cnt).sum(0) / n
    m2 = ((var_all.double() + (mean_all.double() - mean) ** 2) * cnt).sum(0)
    var_b = m2 / n
    var_u = m2 / (n - 1)
    inv_std = 1.0 / torch.sqrt(var_b + eps)
    return mean.float(), var_u.float(), inv_std.float()


def _torch_bn(x, mean, inv_std, weight, bias, channel_last, z=None, fuse_relu=False):
    shp = _bshape(x, channel_last)
    y = (x.float() - mean.view(shp)) * inv_std.view(shp)
    if weight is not None:
        y = y * weight.float().view(shp)
    if bias is not None:
        y = y + bias.float().view(shp)
    if z is not None:
        y = y + z.float()
    if fuse_relu:
        y = torch.relu(y)
    return y


def batchnorm_forward(x, mean, inv_std, weight, bias, channel_last=False, z=None, fuse_relu=False):
    if _native.use_native(x):
        m = _syncbn()
        x = x.contiguous()
        if channel_last:
            return m.batchnorm_forward_c_last(x, _c(z), mean, inv_std, weight, bias, fuse_relu)
        if z is not None or fuse_relu:
            y = m.batchnorm_forward(x, mean, inv_std, weight, bias)
            if z is not None:
                y = y + z
            return torch.relu_(y) if fuse_relu else y
        return m.batchnorm_forward(x, mean, inv_std, weight, bias)
    return _torch_bn(x, mean, inv_std, weight, bias, channel_last, z, fuse_relu).to(x.dtype)


def relu_backward(grad_out, x, z, mean, inv_std, weight, bias, channel_last=True):
    """Mask the incoming grad by the recomputed fused-ReLU output (materialized; needed when the
    residual input ``z`` requires a gradient)."""
    if _native.use_native(x) and channel_last:
        return _syncbn().relu_bw_c_last(grad_out.contiguous(), x.contiguous(), _c(z), mean, inv_std, weight, bias)
    y = _torch_bn(x, mean, inv_std, weight, bias, channel_last, z, False)
    return torch.where(y > 0, grad_out, torch.zeros_like(grad_out))


def reduce_bn(grad_out, x, mean, inv_std, weight, channel_last=False, z=None, bias=None, fuse_relu=False):
    """Returns (sum_dy, sum_dy_xmu, grad_weight, grad_bias) over the local batch.  With
    ``fuse_relu`` the grad is first masked by relu(bn(x)+z) > 0 (recomputed in-kernel)."""
    if _native.use_native(x):
        m = _syncbn()
        x = x.contiguous()
        if channel_last:
            return tuple(m.reduce_bn_c_last(grad_out, x, mean, inv_std, weight, _c(z), bias, fuse_relu))
        if fuse_relu:
            grad_out = relu_backward(grad_out, x, z, mean, inv_std, weight, bias, False)
        return tuple(m.reduce_bn(grad_out.contiguous(), x, mean, inv_std, weight))
    if fuse_relu:
        grad_out = relu_backward(grad_out, x, z, mean, inv_std, weight, bias, channel_last)
    shp = _bshape(x, channel_last)
    dims = _reduce_dims(x, channel_last)
    dy = grad_out.float()
    xmu = x.float() - mean.view(shp)
    sum_dy = dy.sum(dims)
    sum_dy_xmu = (dy * xmu).sum(dims)
    gw = sum_dy_xmu * inv_std if weight is not None else None
    gb = sum_dy if weight is not None else None
    if weight is not None:
        gw = gw.to(weight.dtype)
        gb = gb.to(weight.dtype)
    return sum_dy, sum_dy_xmu, gw, gb


def batchnorm_backward(grad_out, x, mean, inv_std, weight, sum_dy, sum_dy_xmu, count, channel_last=False, z=None,
                       bias=None, fuse_relu=False):
    """dx given the (globally reduced) sums; ``count`` = per-rank element counts [world]."""
    if _native.use_native(x):
        m = _syncbn()
        c = count.to(torch.int32)
        x = x.contiguous()
        if channel_last:
            return m.batchnorm_backward_c_last(grad_out, x, mean, inv_std, weight, sum_dy, sum_dy_xmu, c, _c(z), bias,
                                               fuse_relu)
        if fuse_relu:
            grad_out = relu_backward(grad_out, x, z, mean, inv_std, weight, bias, False)
        return m.batchnorm_backward(grad_out.contiguous(), x, mean, inv_std, weight, sum_dy, sum_dy_xmu, c)
    if fuse_relu:
        grad_out = relu_backward(grad_out, x, z, mean, inv_std, weight, bias, channel_last)
    shp = _bshape(x, channel_last)
    n = float(count.sum())
    dy = grad_out.float()
    xmu = x.float() - mean.view(shp)
    istd = inv_std.view(shp)
    w = weight.float().view(shp) if weight is not None else 1.0
    mean_dy = (sum_dy / n).view(shp)
    mean_dy_xmu = (sum_dy_xmu / n).view(shp)
    dx = (dy - mean_dy - xmu * istd * istd * mean_dy_xmu) * istd * w
    return dx.to(x.dtype)
