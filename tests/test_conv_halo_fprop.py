"""Halo-tile 3x3 stride-1 convolution (csrc/conv/conv3x3_halo.hip, the default conv_tap_fprop
engine for C % 64 == 0, K % 128 == 0): forward (+ BN statistics epilogue), the flipped-weight
data gradient and the BN + ReLU operand prologue, against a float64 torch reference of the same
bf16 / fp16 operands.  Shapes cover tiles that cross image boundaries (the padded row space), a
ragged last tile, several tiles per workgroup, and small images with many images per tile."""
import pytest
import torch
import torch.nn.functional as F

@pytest.fixture(autouse=True)
def _halo_everywhere():
    """Route every supported shape to the halo-tile kernel (the default takes it at <= 64-pixel
    images only), then restore the default."""
    import apex

    if not torch.cuda.is_available():
        yield
        return
    ext = apex._native.require("conv").conv
    ext.hfp_set_mode(2)
    yield
    ext.hfp_set_mode(-1)


SHAPES = [
    # n, h, w, cin, cout
    (3, 28, 28, 128, 128),
    (2, 14, 14, 256, 256),
    (5, 7, 7, 128, 256),
    (2, 9, 13, 64, 128),
    (1, 40, 6, 192, 128),
    (4, 5, 5, 64, 384),
    (2, 56, 56, 128, 128),
]


def _close(a, b, tol):
    scale = max(1.0, float(b.abs().max()))
    err = float((a.double().cpu() - b).abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,cin,cout", SHAPES)
def test_gpu_halo_fprop_dgrad_stats(dtype, n, h, w, cin, cout):
    from apex import _native
    from apex.ops import conv as C

    ext = _native.require("conv").conv
    assert ext.hfp_supported(n, h, w, cin, cout), "shape expected on the halo-tile kernel"
    torch.manual_seed(h * 7 + w + cin)
    x = (torch.randn(n, cin, h, w, device="cuda") + 0.1).to(dtype).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.05).to(dtype).contiguous(memory_format=torch.channels_last)
    xd, wd = x.double().cpu(), wt.double().cpu()
    ref = F.conv2d(xd, wd, None, 1, 1)
    y = C.conv_tap_forward(x, wt, 1, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    _close(y, ref, 1e-2)
    shift = torch.randn(cout, device="cuda") * 0.1
    y2, part = C.conv_tap_forward(x, wt, 1, 1, stats_shift=shift)
    assert torch.equal(y2, y)
    yf = y2.double().cpu().permute(0, 2, 3, 1).reshape(-1, cout)
    s1 = part[0].double().cpu().sum(0)
    s2 = part[1].double().cpu().sum(0)
    sd = shift.double().cpu()
    torch.testing.assert_close(s1, (yf - sd).sum(0), atol=1e-3 * yf.numel() ** 0.5, rtol=1e-4)
    torch.testing.assert_close(s2, ((yf - sd) ** 2).sum(0), atol=1e-3, rtol=1e-4)
    # data gradient: the same kernel over dY with the flipped, transposed weight (C % 128 needed)
    if cin % 128 == 0:
        gy = torch.randn(n, cout, h, w, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
        xr = xd.clone().requires_grad_(True)
        torch.autograd.backward(F.conv2d(xr, wd, None, 1, 1), gy.double().cpu())
        dx = C.conv_tap_dgrad(gy, wt, x.shape, 1, 1)
        _close(dx, xr.grad, 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,cin,cout", [(3, 28, 28, 128, 128), (5, 7, 7, 64, 128), (2, 9, 13, 192, 256)])
def test_gpu_halo_fprop_bn_relu_prologue(n, h, w, cin, cout):
    """relu(x * scale + shift) applied to the staged halo: matches the conv of the explicitly
    normalized input, and the zero padding stays zero (a relu(shift) border would show at every
    image edge)."""
    from apex.ops import conv as C

    torch.manual_seed(11)
    x = torch.randn(n, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    sc = torch.rand(cin, device="cuda") + 0.5
    sh = torch.randn(cin, device="cuda") * 0.5 + 0.3  # positive shifts: relu(shift) != 0 at the padding
    pcoef = torch.cat([sc, sh]).contiguous()
    y = C.conv_tap_forward(x, wt, 1, 1, pcoef=pcoef)
    z = torch.relu(x.float() * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)).to(torch.bfloat16)
    ref = F.conv2d(z.double().cpu(), wt.double().cpu(), None, 1, 1)
    _close(y, ref, 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 56, 56), (3, 17, 40)])
def test_gpu_spatial_fprop_bn_relu_prologue_is_bitwise_the_apply_pass(n, h, w):
    """The 64 -> 64 spatial-tile forward (conv3x3_sp.hip) with the producing BN + ReLU applied to its
    register-staged halo (padding taps stay zero) is BITWISE the forward of the materialised
    apply-pass output, statistics epilogue included."""
    import apex
    from apex.ops import conv as C

    apex._native.require("conv").conv.hfp_set_mode(0)  # the spatial kernel's route, not the halo-tile one
    bn = apex._native.require("bn_nhwc").bn_nhwc
    torch.manual_seed(h)
    dt = torch.bfloat16
    y = torch.randn(n, 64, h, w, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).to(dt).contiguous(memory_format=torch.channels_last)
    coef = torch.cat([torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.5])
    z = bn.apply(y.permute(0, 2, 3, 1).reshape(-1, 64), None, coef, True)[0]
    zv = z.view(n, h, w, 64).permute(0, 3, 1, 2)
    shift = torch.randn(64, device="cuda") * 0.1
    want, wpart = C.conv_tap_forward(zv, wt, 1, 1, stats_shift=shift)
    got, gpart = C.conv_tap_forward(y, wt, 1, 1, stats_shift=shift, pcoef=coef)
    assert torch.equal(got, want) and torch.equal(gpart, wpart)
    ref = F.conv2d(zv.double().cpu(), wt.double().cpu(), None, 1, 1)
    _close(got, ref, 1e-2)
