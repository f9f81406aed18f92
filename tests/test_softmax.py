"""Fused scale/mask/softmax numerics (model: reference tests/L0/run_transformer/test_fused_softmax.py —
fused kernel vs torch softmax, fp16/bf16, padding and causal masks).  GPU tests compare the gfx950
kernels against an fp32 torch reference; CPU tests cover the module's torch path."""
import pytest
import torch

from apex.transformer.enums import AttnMaskType
from apex.transformer.functional import FusedScaleMaskSoftmax
from apex.transformer.functional.fused_softmax import (scaled_masked_softmax, scaled_softmax,
                                                       scaled_upper_triang_masked_softmax)


def attention_mask_func(attention_scores, attention_mask):
    return attention_scores.masked_fill(attention_mask, -10000.0)


def _ref(x, mask, scale, causal):
    xf = x.float() * scale
    if mask is not None:
        xf = xf.masked_fill(mask.bool(), -10000.0)
    if causal:
        sq, sk = xf.shape[-2:]
        xf = xf.masked_fill(torch.ones(sq, sk, dtype=torch.bool, device=x.device).triu(1), float("-inf"))
    return torch.softmax(xf, -1)


def test_cpu_module_paths():
    torch.manual_seed(0)
    x = torch.randn(2, 4, 8, 32).bfloat16()
    mask = torch.randint(0, 2, (2, 1, 8, 32)).bool()
    for mt in (AttnMaskType.padding, AttnMaskType.causal):
        m = FusedScaleMaskSoftmax(False, True, mt, True, attention_mask_func, True, 0.5)
        xx = torch.randn(2, 4, 32, 32).bfloat16() if mt == AttnMaskType.causal else x
        y = m(xx, mask if mt == AttnMaskType.padding else None)
        ref = _ref(xx, mask if mt == AttnMaskType.padding else None, 0.5, mt == AttnMaskType.causal)
        torch.testing.assert_close(y.float(), ref, atol=1e-2, rtol=1e-2)


SKS = [32, 128, 512, 1000, 1024, 2048, 3072, 4096, 8192, 16384, 20000]


@pytest.mark.gpu
@pytest.mark.parametrize("sk", SKS)
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("pad_batches", [1, 2])
def test_gpu_scaled_masked_softmax(sk, dtype, pad_batches):
    torch.manual_seed(sk)
    b, np_, sq = 2, 3, 5
    x = (torch.randn(b, np_, sq, sk, device="cuda") * 4).to(dtype).requires_grad_(True)
    mask = torch.rand(pad_batches, 1, sq, sk, device="cuda") < 0.3
    y = scaled_masked_softmax(x, mask, 0.7)
    xr = x.detach().float().requires_grad_(True)
    yr = _ref(xr, mask, 0.7, False)
    torch.testing.assert_close(y.float(), yr, atol=4e-3, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-2, rtol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("sq", [16, 128, 1000, 2048, 4096])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gpu_causal_softmax(sq, dtype):
    torch.manual_seed(sq)
    x = (torch.randn(1, 2, sq, sq, device="cuda") * 3).to(dtype).requires_grad_(True)
    y = scaled_upper_triang_masked_softmax(x, None, 0.125)
    assert torch.all(y.float().triu(1) == 0)
    xr = x.detach().float().requires_grad_(True)
    yr = _ref(xr, None, 0.125, True)
    torch.testing.assert_close(y.float(), yr, atol=4e-3, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-2, rtol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("sk", [64, 2048, 5000])
def test_gpu_scaled_softmax_fp32(sk):
    x = torch.randn(7, 9, sk, device="cuda", requires_grad=True)
    y = scaled_softmax(x, 1.3)
    xr = x.detach().clone().requires_grad_(True)
    yr = torch.softmax(xr * 1.3, -1)
    torch.testing.assert_close(y, yr, atol=1e-6, rtol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-5, rtol=1e-4)


@pytest.mark.gpu
def test_gpu_module_uses_fused_kernel_beyond_2048():
    m = FusedScaleMaskSoftmax(False, True, AttnMaskType.padding, True, attention_mask_func, True, 1.0)
    assert m.is_kernel_available(torch.zeros(1), 2, 4, 8, 4096)
