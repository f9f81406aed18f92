"""NHWC max pool (gfx950 kernel) vs F.max_pool2d on the same channels_last input."""
import pytest
import torch
import torch.nn.functional as F

from apex.ops.pooling import MaxPool2dNHWC, max_pool2d_nhwc


def test_cpu_falls_back_to_torch():
    x = torch.randn(2, 16, 9, 9).to(memory_format=torch.channels_last)
    torch.testing.assert_close(MaxPool2dNHWC(3, 2, 1)(x), F.max_pool2d(x, 3, 2, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 112, 112), 3, 2, 1), ((2, 32, 15, 17), 3, 2, 1),
                                          ((2, 16, 8, 8), 2, 2, 0), ((1, 8, 9, 7), 3, 1, 1)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_gpu_maxpool_nhwc(shape, k, s, p, dtype):
    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dtype).to(memory_format=torch.channels_last).requires_grad_(True)
    xr = x.detach().clone().requires_grad_(True)
    y = max_pool2d_nhwc(x, k, s, p)
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y, yr, atol=0, rtol=0)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    # ties (equal maxima) could route gradient differently; random data has none
    torch.testing.assert_close(x.grad.float(), xr.grad.float(), atol=1e-2 if dtype != torch.float32 else 1e-5,
                               rtol=1e-2)
