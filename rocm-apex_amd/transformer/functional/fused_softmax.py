"""Fused scale + mask + softmax (reference apex/transformer/functional/fused_softmax.py:21-199).

GPU: gfx950 kernels in ``csrc/softmax/softmax.hip`` (register-resident rows of up to 16384 keys;
the reference's kernels stop at 2048).  CPU: the same math in torch (fp32 accumulation), so the
module works in the CPU test tier."""
import torch

from ... import _native
from ..._autocast_utils import _autocast_disabled, _cast_if_autocast_enabled
from ..enums import AttnMaskType

MAX_FUSED_KEYS = 16384


def _ext(name):
    return getattr(_native.require(name), name)


def _torch_softmax_fwd(x, mask, scale, causal):
    xf = x.float() * scale
    if mask is not None:
        xf = xf.masked_fill(mask.bool(), -10000.0)
    if causal:
        sq, sk = xf.shape[-2], xf.shape[-1]
        tri = torch.ones(sq, sk, dtype=torch.bool, device=x.device).triu(1)
        xf = xf.masked_fill(tri, float("-inf"))
    return torch.softmax(xf, dim=-1).to(x.dtype)


def _torch_softmax_bwd(g, y, scale):
    gf, yf = g.float(), y.float()
    return (scale * yf * (gf - (gf * yf).sum(-1, keepdim=True))).to(y.dtype)


class ScaledUpperTriangMaskedSoftmax(torch.autograd.Function):
    """Causal (upper-triangular) mask; input [attn_batches, sq, sk] with sq == sk."""

    @staticmethod
    def forward(ctx, inputs, scale):
        if _native.use_native(inputs):
            y = _ext("scaled_upper_triang_masked_softmax_cuda").forward(inputs, float(scale))
        else:
            y = _torch_softmax_fwd(inputs, None, scale, True)
        ctx.scale = float(scale)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, output_grads):
        (y,) = ctx.saved_tensors
        if _native.use_native(y):
            return _ext("scaled_upper_triang_masked_softmax_cuda").backward(output_grads, y, ctx.scale), None
        return _torch_softmax_bwd(output_grads, y, ctx.scale), None


def scaled_upper_triang_masked_softmax(inputs, _, scale):
    b, np_, sq, sk = inputs.size()
    assert sq == sk, "causal mask is only for self attention"
    inputs = inputs.view(-1, sq, sk)
    args = _cast_if_autocast_enabled(inputs, scale)
    with _autocast_disabled():
        probs = ScaledUpperTriangMaskedSoftmax.apply(*args)
    return probs.view(b, np_, sq, sk)


class ScaledMaskedSoftmax(torch.autograd.Function):
    """Padding mask ([b or 1, 1, sq, sk], nonzero == masked -> -10000)."""

    @staticmethod
    def forward(ctx, inputs, mask, scale):
        if _native.use_native(inputs):
            y = _ext("scaled_masked_softmax_cuda").forward(inputs, mask, float(scale))
        else:
            y = _torch_softmax_fwd(inputs, mask, scale, False)
        ctx.scale = float(scale)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, output_grads):
        (y,) = ctx.saved_tensors
        if _native.use_native(y):
            return _ext("scaled_masked_softmax_cuda").backward(output_grads, y, ctx.scale), None, None
        return _torch_softmax_bwd(output_grads, y, ctx.scale), None, None


def scaled_masked_softmax(inputs, mask, scale):
    args = _cast_if_autocast_enabled(inputs, mask, scale)
    with _autocast_disabled():
        return ScaledMaskedSoftmax.apply(*args)


class ScaledSoftmax(torch.autograd.Function):
    """No mask: softmax(scale * x) over the last dim."""

    @staticmethod
    def forward(ctx, inputs, scale):
        if _native.use_native(inputs):
            y = _ext("scaled_softmax_cuda").forward(inputs, float(scale))
        else:
            y = _torch_softmax_fwd(inputs, None, scale, False)
        ctx.scale = float(scale)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, output_grads):
        (y,) = ctx.saved_tensors
        if _native.use_native(y):
            return _ext("scaled_softmax_cuda").backward(output_grads, y, ctx.scale), None
        return _torch_softmax_bwd(output_grads, y, ctx.scale), None


def scaled_softmax(inputs, scale):
    args = _cast_if_autocast_enabled(inputs, scale)
    with _autocast_disabled():
        return ScaledSoftmax.apply(*args)


class FusedScaleMaskSoftmax(torch.nn.Module):
    """fused operation: scaling + mask + softmax (reference :95-199).

    Arguments: input_in_fp16, input_in_bf16, attn_mask_type (padding / causal),
    scaled_masked_softmax_fusion, mask_func, softmax_in_fp32, scale."""

    def __init__(self, input_in_fp16, input_in_bf16, attn_mask_type, scaled_masked_softmax_fusion, mask_func,
                 softmax_in_fp32, scale):
        super().__init__()
        self.input_in_fp16 = input_in_fp16
        self.input_in_bf16 = input_in_bf16
        if self.input_in_fp16 and self.input_in_bf16:
            raise RuntimeError("both fp16 and bf16 flags cannot be active at the same time.")
        self.input_in_float16 = self.input_in_fp16 or self.input_in_bf16
        self.attn_mask_type = attn_mask_type
        self.scaled_masked_softmax_fusion = scaled_masked_softmax_fusion
        self.mask_func = mask_func
        self.softmax_in_fp32 = softmax_in_fp32
        self.scale = scale
        if not (self.scale is None or softmax_in_fp32):
            raise RuntimeError("softmax should be in fp32 when scaled")
        if self.scaled_masked_softmax_fusion:
            if self.attn_mask_type == AttnMaskType.causal:
                self.fused_softmax_func = scaled_upper_triang_masked_softmax
            elif self.attn_mask_type == AttnMaskType.padding:
                self.fused_softmax_func = scaled_masked_softmax
            else:
                raise ValueError("Invalid attn_mask_type.")

    def forward(self, input, mask):
        assert input.dim() == 4  # [b, np, sq, sk]
        if self.is_kernel_available(mask, *input.size()):
            return self.forward_fused_softmax(input, mask)
        return self.forward_torch_softmax(input, mask)

    def is_kernel_available(self, mask, b, np, sq, sk):
        if not (self.scaled_masked_softmax_fusion and self.input_in_float16 and 0 < sk <= MAX_FUSED_KEYS):
            return False
        if self.attn_mask_type == AttnMaskType.causal:
            return sq == sk
        return mask is not None

    def forward_fused_softmax(self, input, mask):
        scale = self.scale if self.scale is not None else 1.0
        return self.fused_softmax_func(input, mask, scale)

    def forward_torch_softmax(self, input, mask):
        if self.input_in_float16 and self.softmax_in_fp32:
            input = input.float()
        if self.scale is not None:
            input = input * self.scale
        mask_output = self.mask_func(input, mask) if mask is not None else input
        probs = torch.nn.Softmax(dim=-1)(mask_output)
        if self.input_in_float16 and self.softmax_in_fp32:
            probs = probs.half() if self.input_in_fp16 else probs.bfloat16()
        return probs

    @staticmethod
    def get_batch_per_block(sq, sk, b, np):
        return 1
