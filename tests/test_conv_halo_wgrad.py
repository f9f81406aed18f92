"""Halo-tile 3x3 stride-1 weight gradient (csrc/conv/conv3x3_wgrad.hip, the default conv_wgrad
engine where it applies) against a float64 torch reference of the same bf16 / fp16 operands:
every ResNet-50 stage geometry (rows-of-one-image tiles at 56 / 28 / 14, two whole images per
tile at 7 with an odd batch: a partial last tile), ragged widths and small images, fp32 and
16-bit outputs."""
import pytest
import torch
import torch.nn.functional as F

SHAPES = [
    # n, h, w, cin, cout
    (2, 56, 56, 64, 64),
    (2, 28, 28, 128, 128),
    (3, 14, 14, 256, 128),
    (3, 7, 7, 512, 64),
    (2, 12, 12, 64, 128),
    (3, 9, 9, 128, 64),
    (5, 5, 5, 64, 64),
    (2, 3, 3, 64, 64),
    (2, 10, 13, 64, 64),
    (1, 30, 17, 64, 192),
]


def _ref(x, gy, cout, stride=1):
    """float64 weight gradient on the CPU (exact products of the 16-bit operands)."""
    xd = x.detach().double().cpu().requires_grad_(False)
    gd = gy.detach().double().cpu()
    w = torch.zeros(cout, x.size(1), 3, 3, dtype=torch.float64, requires_grad=True)
    torch.autograd.backward(F.conv2d(xd, w, None, stride, 1), gd)
    return w.grad


def _close(a, b, tol):
    scale = max(1.0, float(b.abs().max()))
    err = float((a.double().cpu() - b).abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,cin,cout", SHAPES)
def test_gpu_halo_wgrad_matches_float64(dtype, n, h, w, cin, cout):
    from apex import _native
    from apex.ops import conv as C

    ext = _native.require("conv").conv
    assert ext.halo_wgrad_supported(n, h, w, cin, cout), "shape expected on the halo kernel"
    torch.manual_seed(h * 31 + w + cin)
    x = (torch.randn(n, cin, h, w, device="cuda") + 0.1).to(dtype).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, cout, h, w, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    ref = _ref(x, gy, cout)
    ext.force_wgrad_variant(ext.WGRAD_HALO)
    try:
        dw32 = C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 1, 1, torch.float32)
        dw16 = C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 1, 1, dtype)
        again = C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 1, 1, torch.float32)
    finally:
        ext.force_wgrad_variant(-1)
    assert dw32.shape == (cout, cin, 3, 3) and dw32.is_contiguous(memory_format=torch.channels_last)
    _close(dw32, ref, 2e-5)
    _close(dw16, ref, 8e-3)
    assert torch.equal(dw32, again), "split partials must be summed in a fixed order"


@pytest.mark.gpu
def test_gpu_halo_wgrad_is_the_default_route():
    """tap_route sends the ResNet-50 stride-1 3x3 weight gradients to the native path and the
    conv_wgrad dispatcher picks the halo kernel (bitwise the forced variant)."""
    from apex import _native
    from apex.ops import conv as C

    ext = _native.require("conv").conv
    for h, c in ((56, 64), (28, 128), (14, 256), (7, 512)):
        assert C.tap_route(c, c, 3, 1, h, h)[2], (h, c)
    torch.manual_seed(3)
    x = torch.randn(2, 64, 20, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 20, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dflt = C.conv_tap_wgrad(gy, x, (64, 64, 3, 3), 1, 1, torch.float32)
    ext.force_wgrad_variant(ext.WGRAD_HALO)
    try:
        forced = C.conv_tap_wgrad(gy, x, (64, 64, 3, 3), 1, 1, torch.float32)
    finally:
        ext.force_wgrad_variant(-1)
    assert torch.equal(dflt, forced)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 56, 56, 64, 64), (2, 28, 28, 128, 128), (3, 7, 7, 512, 64),
                                            (2, 10, 13, 64, 64)])
def test_gpu_halo_wgrad_bn_relu_prologue_is_bitwise_the_apply_pass(n, h, w, cin, cout):
    """x' = relu(x * xcoef[c] + xcoef[C + c]) recomputed on the halo kernel's staged input (each lane
    rewrites the chunks it loaded; padding stays zero) gives BITWISE the weight gradient of the
    materialised apply-pass output (the same fma / max / rounding)."""
    import apex
    from apex.ops import conv as C

    bn = apex._native.require("bn_nhwc").bn_nhwc
    torch.manual_seed(h + cin)
    dt = torch.bfloat16
    y = torch.randn(n, cin, h, w, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, cout, h, w, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    coef = torch.cat([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.5])
    z = bn.apply(y.permute(0, 2, 3, 1).reshape(-1, cin), None, coef, True)[0]
    zv = z.view(n, h, w, cin).permute(0, 3, 1, 2)
    want = C.conv_tap_wgrad(gy, zv, (cout, cin, 3, 3), 1, 1, torch.float32)
    got = C.conv_tap_wgrad(gy, y, (cout, cin, 3, 3), 1, 1, torch.float32, xcoef=coef)
    assert torch.equal(got, want)
    _close(got, _ref(zv, gy, cout), 1e-2)


# stride 2 over even-sized inputs (n, input h, input w, cin, cout): ResNet-50's three downsampling
# 3x3s (56 -> 28 on 2-row tiles, 8 and 4 waves; 28 -> 14 on 2-row tiles, 8 waves, or 7-row tiles,
# 4 waves; 14 -> 7 as two whole images per tile with an odd batch, 4 waves, or one image per tile,
# 8 waves), a 5-row tile, one whole non-square image per tile, a tiny image
SHAPES_S2 = [
    (2, 56, 56, 128, 128),
    (2, 56, 56, 128, 64),
    (3, 28, 28, 256, 128),
    (3, 28, 28, 256, 64),
    (3, 14, 14, 512, 64),
    (3, 14, 14, 256, 128),
    (2, 20, 20, 64, 64),
    (2, 12, 16, 64, 128),
    (3, 4, 4, 64, 64),
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,h,w,cin,cout", SHAPES_S2)
def test_gpu_halo_wgrad_stride2_matches_float64(dtype, n, h, w, cin, cout):
    """the stride-2 form (2R + 1 halo rows, even / odd column planes) against float64 torch"""
    from apex import _native
    from apex.ops import conv as C

    ext = _native.require("conv").conv
    assert ext.halo_wgrad_supported(n, h, w, cin, cout, 2), "shape expected on the halo kernel"
    torch.manual_seed(h * 17 + w + cin)
    x = (torch.randn(n, cin, h, w, device="cuda") + 0.1).to(dtype).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, cout, h // 2, w // 2, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    ref = _ref(x, gy, cout, 2)
    ext.force_wgrad_variant(ext.WGRAD_HALO)
    try:
        dw32 = C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 2, 1, torch.float32)
        dw16 = C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 2, 1, dtype)
        again = C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 2, 1, torch.float32)
    finally:
        ext.force_wgrad_variant(-1)
    _close(dw32, ref, 2e-5)
    _close(dw16, ref, 8e-3)
    assert torch.equal(dw32, again), "split partials must be summed in a fixed order"
    # the default dispatcher takes the same kernel
    assert torch.equal(C.conv_tap_wgrad(gy, x, (cout, cin, 3, 3), 2, 1, torch.float32), dw32)


def test_halo_wgrad_stride2_route():
    """ResNet-50's downsampling 3x3 weight gradients route to the native kernel when the
    extension takes their shapes (the stride-2 form), MIOpen otherwise."""
    from apex import _native
    from apex.ops import conv as C

    ext = _native.submodule("conv")
    for h, c in ((56, 128), (28, 256), (14, 512)):
        want = bool(ext is not None and C._HALO_WGRAD and C._HALO_WGRAD_S2
                    and ext.halo_wgrad_supported(1, h, h, c, c, 2))
        assert C.tap_route(c, c, 3, 2, h, h)[2] == want
    if ext is not None:
        assert not ext.halo_wgrad_supported(1, 15, 15, 64, 64, 2), "odd inputs stay on the other engines"
