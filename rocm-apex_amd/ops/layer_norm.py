"""LayerNorm / RMSNorm forward+backward entry points (reference csrc/layer_norm_cuda.cpp:121-266).

GPU: gfx950 kernels in ``csrc/norm`` (one wave64 per row, Welford in registers, fp32 stats;
two-stage dgamma/dbeta).  CPU: torch reference.  Shapes: input [n1, n2] flattened from
``input.shape[:-len(normalized_shape)]`` x ``normalized_shape``."""
import torch

from .. import _native


def _norm():
    return _native.require("fused_layer_norm").fused_layer_norm_cuda


def compute_n1_n2(x, normalized_shape):
    n2 = 1
    for s in normalized_shape:
        n2 *= s
    return x.numel() // n2, n2


def ln_fwd(x, normalized_shape, weight, bias, eps, rms=False, out_dtype=None):
    """Returns (y, mean, invvar); mean is None for RMSNorm."""
    if _native.use_native(x):
        m = _norm()
        if rms:
            y, invvar = m.rms_forward_affine(x, list(normalized_shape), weight, eps, out_dtype) if weight is not None \
                else m.rms_forward(x, list(normalized_shape), eps)
            return y, None, invvar
        if weight is not None:
            y, mean, invvar = m.forward_affine(x, list(normalized_shape), weight, bias, eps, out_dtype)
        else:
            y, mean, invvar = m.forward(x, list(normalized_shape), eps)
        return y, mean, invvar
    n1, n2 = compute_n1_n2(x, normalized_shape)
    xf = x.float().reshape(n1, n2)
    if rms:
        invvar = torch.rsqrt((xf * xf).mean(1) + eps)
        y = xf * invvar[:, None]
        mean = None
    else:
        mean = xf.mean(1)
        var = xf.var(1, unbiased=False)
        invvar = torch.rsqrt(var + eps)
        y = (xf - mean[:, None]) * invvar[:, None]
    if weight is not None:
        y = y * weight.float().reshape(1, n2)
    if bias is not None:
        y = y + bias.float().reshape(1, n2)
    od = out_dtype if out_dtype is not None else x.dtype
    return y.reshape(x.shape).to(od), mean, invvar


def ln_bwd(dy, x, mean, invvar, normalized_shape, weight, bias, eps, rms=False, dres=None):
    """Returns (dx, dgamma, dbeta) (dgamma/dbeta None when weight is None).  ``dres``: a gradient
    added to dx (the residual branch's, summed inside the affine LayerNorm kernel on the GPU)."""
    if dres is not None and not (_native.use_native(x) and not rms and weight is not None
                                 and dres.dtype == dy.dtype):
        dx, dgamma, dbeta = ln_bwd(dy, x, mean, invvar, normalized_shape, weight, bias, eps, rms)
        return dx + dres.to(dx.dtype).reshape(dx.shape), dgamma, dbeta
    if _native.use_native(x):
        m = _norm()
        if rms:
            if weight is not None:
                dx, dgamma = m.rms_backward_affine(dy, invvar, x, list(normalized_shape), weight, eps)
                return dx, dgamma, None
            return m.rms_backward(dy, invvar, x, list(normalized_shape), eps), None, None
        if weight is not None:
            dx, dgamma, dbeta = m.backward_affine(dy, mean, invvar, x, list(normalized_shape), weight, bias, eps,
                                                  dres=dres)
            return dx, dgamma, (dbeta if bias is not None else None)
        return m.backward(dy, mean, invvar, x, list(normalized_shape), eps), None, None
    n1, n2 = compute_n1_n2(x, normalized_shape)
    xf = x.float().reshape(n1, n2)
    g = dy.float().reshape(n1, n2)
    xhat = (xf - mean[:, None]) * invvar[:, None] if not rms else xf * invvar[:, None]
    w = weight.float().reshape(1, n2) if weight is not None else torch.ones(1, n2, dtype=torch.float32)
    gw = g * w
    if rms:
        dx = invvar[:, None] * (gw - xhat * (gw * xhat).mean(1, keepdim=True))
    else:
        dx = invvar[:, None] * (gw - gw.mean(1, keepdim=True) - xhat * (gw * xhat).mean(1, keepdim=True))
    dgamma = (g * xhat).sum(0).reshape(normalized_shape).to(weight.dtype) if weight is not None else None
    dbeta = g.sum(0).reshape(normalized_shape).to(bias.dtype) if bias is not None else None
    return dx.reshape(x.shape).to(x.dtype), dgamma, dbeta
