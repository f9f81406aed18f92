"""1x1 stride-1 convolution routed to the gfx950 MFMA GEMM (apex.ops.conv) vs fp32 torch conv."""
import pytest
import torch
import torch.nn.functional as F

from apex.ops.conv import Conv1x1NHWC, _Conv1x1Fn, route


def test_cpu_falls_back_and_matches_conv2d_state():
    torch.manual_seed(0)
    m = Conv1x1NHWC(64, 128)
    ref = torch.nn.Conv2d(64, 128, 1, bias=False)
    assert list(m.state_dict()) == list(ref.state_dict())
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 64, 5, 5).to(memory_format=torch.channels_last)
    torch.testing.assert_close(m(x), ref(x))


def test_route_policy():
    # ResNet-50 bs 256, per-op winners of profiles/conv_routes_ab_r03.jsonl
    assert route(256 * 7 * 7, 2048, 512) == ("lib", "lib", "native")
    assert route(256 * 7 * 7, 512, 2048) == ("native", "lib", "native")
    assert route(256 * 14 * 14, 1024, 256) == ("lib", "lib", "native")
    assert route(256 * 28 * 28, 512, 256) == ("lib", "lib", "native")
    assert route(256 * 28 * 28, 512, 128) == ("lib", "lib", "miopen")
    assert route(256 * 56 * 56, 64, 256) == ("lib", "miopen", "miopen")
    assert route(256 * 56 * 56, 256, 64) == ("miopen", "lib", "miopen")
    assert route(256 * 56 * 56, 64, 64) == ("miopen", "miopen", "miopen")


def _ref(x, w, gy):
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    yr.backward(gy.float())
    return yr, xr.grad, wr.grad


def _close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    scale = max(1.0, b.abs().max().item())
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,cout,hw", [(4, 1024, 256, 14), (2, 512, 2048, 7), (8, 2048, 512, 7),
                                           (2, 256, 64, 9)])
@pytest.mark.parametrize("routes", [("native", "native", "native"), ("lib", "lib", "native"),
                                    ("miopen", "miopen", "native"), ("lib", "native", "miopen"),
                                    ("native", "miopen", "miopen")])
def test_gpu_conv1x1_native(n, cin, cout, hw, routes):
    from apex import _native

    assert _native.available(), "native extension must be loaded on a GPU box"
    torch.manual_seed(0)
    dt = torch.bfloat16
    x = torch.randn(n, cin, hw, hw, device="cuda", dtype=dt).to(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(dt)
    gy = torch.randn(n, cout, hw, hw, device="cuda", dtype=dt).to(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    wa = w.clone().requires_grad_(True)
    y = _Conv1x1Fn.apply(xa, wa, routes)
    assert y.is_contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    yr, dxr, dwr = _ref(x, w, gy)
    _close(y, yr)
    _close(xa.grad, dxr)
    _close(wa.grad, dwr)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.gpu
def test_gpu_conv1x1_module_routes_native_backward():
    torch.manual_seed(0)
    m = Conv1x1NHWC(512, 2048).cuda().to(torch.bfloat16)
    x = torch.randn(4, 512, 7, 7, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    assert m._native_ok(x)
    y = m(x)
    assert y.grad_fn is not None and "Conv1x1Fn" in type(y.grad_fn).__name__
    gy = torch.randn_like(y)
    y.backward(gy)
    yr, dxr, dwr = _ref(x, m.weight, gy)
    _close(y, yr)
    _close(x.grad, dxr)
    _close(m.weight.grad, dwr)


def test_channel_pad_conv_cpu_is_plain_conv():
    from apex.ops.conv import ChannelPadConv2d

    torch.manual_seed(0)
    m = ChannelPadConv2d(3, 16, kernel_size=7, stride=2, padding=3, bias=False)
    ref = torch.nn.Conv2d(3, 16, 7, 2, 3, bias=False)
    assert list(m.state_dict()) == list(ref.state_dict())
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 3, 32, 32)
    torch.testing.assert_close(m(x), ref(x))


@pytest.mark.gpu
def test_gpu_channel_pad_stem_matches_conv():
    from apex.ops.conv import ChannelPadConv2d

    torch.manual_seed(0)
    m = ChannelPadConv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False).cuda().to(torch.bfloat16)
    m = m.to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    y = m(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.float()
    wr = m.weight.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 2, 3)
    yr.backward(gy.float())
    _close(y, yr)
    _close(m.weight.grad, wr.grad)
    assert m.weight.grad.shape == (64, 3, 7, 7)
