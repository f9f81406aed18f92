"""gfx950 implicit-GEMM NHWC convolutions (csrc/conv/conv_igemm.hip, apex.ops.conv): forward,
data gradient (stride 1: flipped-weight forward; stride 2: per-phase launches) and weight gradient
against the fp32 PyTorch convolution of the same bf16/fp16 operands."""
import pytest
import torch
import torch.nn.functional as F

SHAPES = [
    # cin, cout, k, stride, h, batch
    (64, 64, 3, 1, 12, 3),
    (128, 64, 3, 1, 9, 2),
    (64, 128, 3, 2, 14, 2),
    (128, 256, 3, 2, 7, 3),
    (256, 256, 3, 1, 7, 5),
    (64, 128, 1, 2, 10, 2),
    (128, 512, 1, 2, 14, 2),
    (192, 320, 3, 1, 5, 7),
]


def _close(a, b, tol):
    scale = max(1.0, float(b.abs().max()))
    err = float((a.float() - b.float()).abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin,cout,k,stride,h,batch", SHAPES)
def test_gpu_conv_tap_fwd_dgrad_wgrad(dtype, cin, cout, k, stride, h, batch):
    import apex
    from apex.ops import conv as C

    torch.manual_seed(0)
    pad = k // 2
    x = torch.randn(batch, cin, h, h, device="cuda").to(dtype).to(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device="cuda") * 0.05).to(dtype).to(memory_format=torch.channels_last)
    y = C.conv_tap_forward(x, w, stride, pad)
    yr = F.conv2d(x.float(), w.float(), None, stride, pad)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    _close(y, yr, 2e-2)
    gy = torch.randn_like(yr).to(dtype).contiguous(memory_format=torch.channels_last)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    torch.autograd.backward(F.conv2d(xr, wr, None, stride, pad), gy.float())
    dx = C.conv_tap_dgrad(gy, w, x.shape, stride, pad)
    _close(dx, xr.grad, 2e-2)
    dw = C.conv_tap_wgrad(gy, x, w.shape, stride, pad, dtype)
    assert dw.shape == w.shape and dw.is_contiguous(memory_format=torch.channels_last)
    _close(dw, wr.grad, 2e-2)
    dw32 = C.conv_tap_wgrad(gy, x, w.shape, stride, pad, torch.float32)
    _close(dw32, wr.grad, 5e-3)


@pytest.mark.gpu
def test_gpu_conv2d_nhwc_module_autograd():
    """Conv2dNHWC: same parameters as nn.Conv2d, native path taken, grads match the torch module."""
    import apex
    from apex.ops import conv as C

    torch.manual_seed(1)
    m = C.Conv2dNHWC(256, 256, 3, stride=2).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    assert C.tap_route(256, 256, 3, 2, 16)[0], "shape expected on the native forward path"
    ref = torch.nn.Conv2d(256, 256, 3, 2, 1, bias=False).cuda()
    ref.weight.data.copy_(m.weight.float())
    x = torch.randn(4, 256, 16, 16, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    calls = {"n": 0}
    orig = C.conv_tap_forward

    def counting(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    C.conv_tap_forward = counting
    try:
        y = m(x)
    finally:
        C.conv_tap_forward = orig
    assert calls["n"] == 1, "native conv path not taken"
    yr = ref(xr)
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)
    _close(y, yr, 2e-2)
    _close(x.grad, xr.grad, 2e-2)
    _close(m.weight.grad, ref.weight.grad, 2e-2)
