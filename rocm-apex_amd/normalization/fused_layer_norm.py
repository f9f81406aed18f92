"""FusedLayerNorm / MixedFusedLayerNorm (+ RMSNorm variants)
(reference apex/normalization/fused_layer_norm.py:15-218).

Autograd functions over :mod:`apex.ops.layer_norm` (gfx950 kernels on GPU).  The "mixed dtypes"
variant returns the output in the dtype of ``weight`` (e.g. bf16 activations with fp32 gamma in
Megatron-style models).  Under ``torch.autocast`` the inputs are cast like ``F.layer_norm``."""
import numbers
import os

import torch
from torch.nn import functional as F
from torch.nn import init
from torch.nn.parameter import Parameter

from .._autocast_utils import _autocast_disabled, _cast_if_autocast_enabled

# APEX_AMD_LN_RESIDUAL=0: layer_norm_with_residual returns the plain pair (A/B switch)
_LN_RESIDUAL = os.environ.get("APEX_AMD_LN_RESIDUAL", "1") != "0"
from ..ops import layer_norm as lnops


def _shape(normalized_shape):
    if isinstance(normalized_shape, numbers.Integral):
        return (normalized_shape,)
    return tuple(normalized_shape)


class FusedLayerNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps, out_dtype=None):
        ctx.normalized_shape = _shape(normalized_shape)
        ctx.eps = eps
        x = input.contiguous()
        w = weight.contiguous()
        b = bias.contiguous() if bias is not None else None
        y, mean, invvar = lnops.ln_fwd(x, ctx.normalized_shape, w, b, eps, out_dtype=out_dtype)
        ctx.save_for_backward(x, w, b, mean, invvar)
        return y

    @staticmethod
    def backward(ctx, grad_output):
        x, w, b, mean, invvar = ctx.saved_tensors
        dx, dw, db = lnops.ln_bwd(grad_output.contiguous(), x, mean, invvar, ctx.normalized_shape, w, b, ctx.eps)
        return dx, dw, db, None, None, None


class FusedLayerNormResidualFunction(torch.autograd.Function):
    """(LN(x), x) as ONE autograd node for a pre-LN residual block, where x feeds both the norm and
    the residual add: backward gets both gradients and the LayerNorm backward kernel returns
    dx = LN'(dy) + d(residual) in the same pass — the autograd sum of the two branches is not a
    separate elementwise kernel (two per transformer layer)."""

    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps):
        ctx.normalized_shape = _shape(normalized_shape)
        ctx.eps = eps
        x = input.contiguous()
        w = weight.contiguous()
        b = bias.contiguous() if bias is not None else None
        y, mean, invvar = lnops.ln_fwd(x, ctx.normalized_shape, w, b, eps)
        ctx.save_for_backward(x, w, b, mean, invvar)
        return y, input.view_as(input)

    @staticmethod
    def backward(ctx, grad_output, grad_residual):
        x, w, b, mean, invvar = ctx.saved_tensors
        dres = grad_residual.contiguous() if grad_residual is not None else None
        dx, dw, db = lnops.ln_bwd(grad_output.contiguous(), x, mean, invvar, ctx.normalized_shape, w, b, ctx.eps,
                                  dres=dres)
        return dx, dw, db, None, None


def layer_norm_with_residual(ln, input):
    """``(ln(input), input)`` with the two branches' gradients summed inside the LayerNorm backward
    when ``ln`` is an affine FusedLayerNorm (else the plain pair: autograd adds them)."""
    if (_LN_RESIDUAL and isinstance(ln, FusedLayerNorm) and ln.elementwise_affine and input.is_cuda
            and not torch.is_autocast_enabled("cuda") and input.dtype == ln.weight.dtype):
        return FusedLayerNormResidualFunction.apply(input, ln.weight, ln.bias, ln.normalized_shape, ln.eps)
    return ln(input), input


class FusedLayerNormAffineMixedDtypesFunction(FusedLayerNormAffineFunction):
    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps):
        return FusedLayerNormAffineFunction.forward(ctx, input, weight, bias, normalized_shape, eps,
                                                    out_dtype=weight.dtype)


class FusedLayerNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, normalized_shape, eps):
        ctx.normalized_shape = _shape(normalized_shape)
        ctx.eps = eps
        x = input.contiguous()
        y, mean, invvar = lnops.ln_fwd(x, ctx.normalized_shape, None, None, eps)
        ctx.save_for_backward(x, mean, invvar)
        return y

    @staticmethod
    def backward(ctx, grad_output):
        x, mean, invvar = ctx.saved_tensors
        dx, _, _ = lnops.ln_bwd(grad_output.contiguous(), x, mean, invvar, ctx.normalized_shape, None, None, ctx.eps)
        return dx, None, None


class FusedRMSNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, normalized_shape, eps, out_dtype=None):
        ctx.normalized_shape = _shape(normalized_shape)
        ctx.eps = eps
        x = input.contiguous()
        w = weight.contiguous()
        y, _, invvar = lnops.ln_fwd(x, ctx.normalized_shape, w, None, eps, rms=True, out_dtype=out_dtype)
        ctx.save_for_backward(x, w, invvar)
        return y

    @staticmethod
    def backward(ctx, grad_output):
        x, w, invvar = ctx.saved_tensors
        dx, dw, _ = lnops.ln_bwd(grad_output.contiguous(), x, None, invvar, ctx.normalized_shape, w, None, ctx.eps,
                                 rms=True)
        return dx, dw, None, None, None


class FusedRMSNormAffineMixedDtypesFunction(FusedRMSNormAffineFunction):
    @staticmethod
    def forward(ctx, input, weight, normalized_shape, eps):
        return FusedRMSNormAffineFunction.forward(ctx, input, weight, normalized_shape, eps, out_dtype=weight.dtype)


class FusedRMSNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, normalized_shape, eps):
        ctx.normalized_shape = _shape(normalized_shape)
        ctx.eps = eps
        x = input.contiguous()
        y, _, invvar = lnops.ln_fwd(x, ctx.normalized_shape, None, None, eps, rms=True)
        ctx.save_for_backward(x, invvar)
        return y

    @staticmethod
    def backward(ctx, grad_output):
        x, invvar = ctx.saved_tensors
        dx, _, _ = lnops.ln_bwd(grad_output.contiguous(), x, None, invvar, ctx.normalized_shape, None, None, ctx.eps,
                                rms=True)
        return dx, None, None


def fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6):
    args = _cast_if_autocast_enabled(input, weight, bias, normalized_shape, eps)
    with _autocast_disabled():
        return FusedLayerNormAffineFunction.apply(*args)


def fused_layer_norm(input, normalized_shape, eps=1e-6):
    args = _cast_if_autocast_enabled(input, normalized_shape, eps)
    with _autocast_disabled():
        return FusedLayerNormFunction.apply(*args)


def mixed_dtype_fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6):
    args = _cast_if_autocast_enabled(input, weight, bias, normalized_shape, eps)
    with _autocast_disabled():
        return FusedLayerNormAffineMixedDtypesFunction.apply(*args)


def fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6):
    args = _cast_if_autocast_enabled(input, weight, normalized_shape, eps)
    with _autocast_disabled():
        return FusedRMSNormAffineFunction.apply(*args)


def fused_rms_norm(input, normalized_shape, eps=1e-6):
    args = _cast_if_autocast_enabled(input, normalized_shape, eps)
    with _autocast_disabled():
        return FusedRMSNormFunction.apply(*args)


def mixed_dtype_fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6):
    args = _cast_if_autocast_enabled(input, weight, normalized_shape, eps)
    with _autocast_disabled():
        return FusedRMSNormAffineMixedDtypesFunction.apply(*args)


class FusedLayerNorm(torch.nn.Module):
    """Drop-in for ``torch.nn.LayerNorm`` backed by the gfx950 kernel."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True):
        super().__init__()
        self.normalized_shape = _shape(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        if self.elementwise_affine:
            self.weight = Parameter(torch.empty(*self.normalized_shape))
            self.bias = Parameter(torch.empty(*self.normalized_shape))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)
            init.zeros_(self.bias)

    def forward(self, input):
        if self.elementwise_affine:
            return fused_layer_norm_affine(input, self.weight, self.bias, self.normalized_shape, self.eps)
        return fused_layer_norm(input, self.normalized_shape, self.eps)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(**self.__dict__)


class FusedRMSNorm(torch.nn.Module):
    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True):
        super().__init__()
        self.normalized_shape = _shape(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        if self.elementwise_affine:
            self.weight = Parameter(torch.empty(*self.normalized_shape))
        else:
            self.register_parameter("weight", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)

    def forward(self, input):
        if self.elementwise_affine:
            return fused_rms_norm_affine(input, self.weight, self.normalized_shape, self.eps)
        return fused_rms_norm(input, self.normalized_shape, self.eps)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(**self.__dict__)


class MixedFusedLayerNorm(FusedLayerNorm):
    """Output dtype follows ``weight`` (reference :202-218)."""

    def __init__(self, normalized_shape, eps=1e-5, **kwargs):
        if "elementwise_affine" in kwargs:
            elementwise_affine = kwargs.pop("elementwise_affine")
            if not elementwise_affine:
                raise RuntimeError("MixedFusedLayerNorm does not support `elementwise_affine = False`")
        super().__init__(normalized_shape=normalized_shape, eps=eps, elementwise_affine=True)

    def forward(self, input):
        return mixed_dtype_fused_layer_norm_affine(input, self.weight, self.bias, self.normalized_shape, self.eps)


class MixedFusedRMSNorm(FusedRMSNorm):
    def __init__(self, normalized_shape, eps=1e-5, **kwargs):
        if "elementwise_affine" in kwargs:
            elementwise_affine = kwargs.pop("elementwise_affine")
            if not elementwise_affine:
                raise RuntimeError("MixedFusedRMSNorm does not support `elementwise_affine = False`")
        super().__init__(normalized_shape=normalized_shape, eps=eps, elementwise_affine=True)

    def forward(self, input):
        return mixed_dtype_fused_rms_norm_affine(input, self.weight, self.normalized_shape, self.eps)
