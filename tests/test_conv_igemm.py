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


CFG_SHAPES = [
    # cin, cout, stride, h, batch: ragged M (not a multiple of 128 / 256), both strides, every
    # output width the configurations tile (64 / 128 / 256 / 512)
    (64, 64, 1, 11, 3),
    (64, 128, 2, 13, 2),
    (128, 256, 1, 9, 3),
    (256, 512, 2, 10, 2),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", list(range(22)))
@pytest.mark.parametrize("cin,cout,stride,h,batch", CFG_SHAPES)
def test_gpu_conv_tap_every_tile_config(cfg, cin, cout, stride, h, batch):
    """Every fprop tile configuration (0-6 fprop_kernel, 7-13 fprop2_kernel: buffer-load staging
    with out-of-range zero fill, 14-20 fprop3, 21 the spatial-tile 64-channel kernel) forced on
    ragged shapes: forward + BN statistics epilogue, the stride-1 / per-phase stride-2 data
    gradient (phase-shifted output placement), and the fused scale / bias / residual / ReLU
    epilogue, against fp32 torch."""
    from apex import _native
    from apex.ops import conv as C

    ext = _native.require("conv").conv
    bn = [128, 64, 128, 64, 128, 64, 256, 64, 64, 128, 128, 128, 256, 256, 64, 64, 128, 128, 128, 256, 64, 64][cfg]
    if cout % bn:
        pytest.skip("tile wider than the output")
    if cfg == 21 and not (cin == 64 and cout == 64 and stride == 1):
        pytest.skip("the spatial-tile kernel is 64 -> 64 channels, stride 1")
    torch.manual_seed(cfg * 7 + cin)
    x = (torch.randn(batch, cin, h, h, device="cuda") + 0.2).to(torch.bfloat16).to(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).to(memory_format=torch.channels_last)
    shift = torch.randn(cout, device="cuda") * 0.1
    C._conv_ext().force_fprop_cfg(cfg)
    try:
        y, part = C.conv_tap_forward(x, w, stride, 1, stats_shift=shift)
        yr = F.conv2d(x.float(), w.float(), None, stride, 1)
        _close(y, yr, 1e-2)
        y2 = yr.permute(0, 2, 3, 1).reshape(-1, cout)
        sm, si, _ = ext.bn_finalize(part, float(y2.size(0)), shift, None, None, None, None, 1e-5, 0.1)
        torch.testing.assert_close(sm, y2.mean(0), atol=3e-3 * float(y2.std()), rtol=2e-3)
        torch.testing.assert_close(si, torch.rsqrt(y2.var(0, unbiased=False) + 1e-5), atol=0, rtol=5e-3)
        # data gradient (its launches run the same fprop kernels with the flipped weight; the
        # stride-2 one places each phase's output with osh = osw = 2)
        if cin % bn == 0:
            gy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            xr = x.float().requires_grad_(True)
            torch.autograd.backward(F.conv2d(xr, w.float(), None, stride, 1), gy.float())
            dx = C.conv_tap_dgrad(gy, w, x.shape, stride, 1)
            _close(dx, xr.grad, 2e-2)
        # fused frozen-BN epilogue: relu(conv * scale + bias + residual)
        if stride == 1:
            sc = torch.rand(cout, device="cuda") + 0.5
            bi = torch.randn(cout, device="cuda") * 0.2
            res = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            out = C.conv_bn_act(x, w, sc, bi, res, True, 1, 1)
            ref = torch.relu(yr * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1) + res.float())
            _close(out, ref, 2e-2)
    finally:
        C._conv_ext().force_fprop_cfg(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", list(range(5)))
@pytest.mark.parametrize("cin,cout,stride,h,batch", CFG_SHAPES + [(128, 128, 1, 7, 5)])
def test_gpu_conv_wgrad_every_variant(variant, cin, cout, stride, h, batch):
    """Every weight-gradient variant (0 wgrad_kernel, 1-4 wgrad2_kernel tiles) forced on ragged
    pixel counts (partial K-steps, zero-filled padding taps) against the fp32 torch gradient."""
    from apex.ops import conv as C

    torch.manual_seed(variant * 11 + cin)
    x = torch.randn(batch, cin, h, h, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, 3, 3, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    ho = (h + 2 - 3) // stride + 1
    gy = torch.randn(batch, cout, ho, ho, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    wr = w.float().requires_grad_(True)
    torch.autograd.backward(F.conv2d(x.float(), wr, None, stride, 1), gy.float())
    C._conv_ext().force_wgrad_variant(variant)
    try:
        dw = C.conv_tap_wgrad(gy, x, w.shape, stride, 1, torch.float32)
        dwb = C.conv_tap_wgrad(gy, x, w.shape, stride, 1, torch.bfloat16)
    finally:
        C._conv_ext().force_wgrad_variant(-1)
    _close(dw, wr.grad, 5e-3)
    _close(dwb, wr.grad, 2e-2)


SP_SHAPES = [
    # n, h, w: ragged in both tile dimensions (8 rows x 32 columns), one tile, the ResNet shape
    (2, 56, 56),
    (3, 9, 33),
    (1, 8, 32),
    (2, 17, 70),
    (5, 3, 5),
]


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", SP_SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_conv_spatial_tile_kernel(n, h, w, dtype):
    """The spatial-tile 3x3 kernel (csrc/conv/conv3x3_sp.hip, the default for 64 -> 64 channels
    stride 1): forward with and without the BN statistics epilogue and the flipped-weight data
    gradient, against fp32 torch, on shapes ragged in both tile dimensions; the statistics rows
    are one per persistent workgroup."""
    from apex import _native
    from apex.ops import conv as C

    ext = _native.require("conv").conv
    torch.manual_seed(h * 131 + w)
    x = (torch.randn(n, 64, h, w, device="cuda") + 0.1).to(dtype).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).to(dtype).contiguous(memory_format=torch.channels_last)
    shift = torch.randn(64, device="cuda") * 0.1
    C._conv_ext().force_fprop_cfg(21)
    try:
        y = C.conv_tap_forward(x, wt, 1, 1)
        yr = F.conv2d(x.float(), wt.float(), None, 1, 1)
        assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
        _close(y, yr, 1e-2)
        y2, part = C.conv_tap_forward(x, wt, 1, 1, stats_shift=shift)
        assert torch.equal(y2, y)
        yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
        sm, si, _ = ext.bn_finalize(part, float(yf.size(0)), shift, None, None, None, None, 1e-5, 0.1)
        torch.testing.assert_close(sm, yf.mean(0), atol=1e-4 * max(1.0, float(yf.std())), rtol=1e-4)
        torch.testing.assert_close(si, torch.rsqrt(yf.var(0, unbiased=False) + 1e-5), atol=0, rtol=1e-3)
        gy = torch.randn_like(yr).to(dtype).contiguous(memory_format=torch.channels_last)
        xr = x.float().requires_grad_(True)
        torch.autograd.backward(F.conv2d(xr, wt.float(), None, 1, 1), gy.float())
        dx = C.conv_tap_dgrad(gy, wt, x.shape, 1, 1)
        _close(dx, xr.grad, 2e-2)
    finally:
        C._conv_ext().force_fprop_cfg(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,h", [(4, 128, 28), (8, 256, 14), (16, 512, 7), (3, 128, 9)])
def test_gpu_dgrad_bn_reduction_epilogue(n, c, h):
    """The stride-1 3x3 data gradient with the producing BN's backward reduction in its epilogue
    (ops/conv.conv_tap_dgrad ``red``): the stored gradient is bitwise the plain dgrad masked by the
    BN's ReLU (recomputed from its input), and the partials sum to the float64 reduction of it."""
    import apex
    from apex.ops import conv as convops

    torch.manual_seed(c + h)
    dt = torch.bfloat16
    gy = torch.randn(n, c, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).to(dt).contiguous(memory_format=torch.channels_last)
    x = torch.randn(n, c, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    coef = torch.cat([torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.3])
    mean = torch.randn(c, device="cuda") * 0.1
    plain = convops.conv_tap_dgrad(gy, w, x.shape, 1, 1)
    dz, part = convops.conv_tap_dgrad(gy, w, x.shape, 1, 1, red=(x, coef, mean))
    mask = (x.float() * coef[:c].view(1, -1, 1, 1) + coef[c:].view(1, -1, 1, 1)) > 0
    want = torch.where(mask, plain, torch.zeros_like(plain))
    assert torch.equal(dz, want)
    g = dz.double().permute(0, 2, 3, 1).reshape(-1, c)
    xm = x.double().permute(0, 2, 3, 1).reshape(-1, c) - mean.double()
    assert part.dim() == 3 and part.size(0) == 2 and part.size(2) == c
    scale = float(g.abs().sum(0).max()) + 1e-6
    torch.testing.assert_close(part[0].double().sum(0), g.sum(0), atol=1e-5 * scale + 1e-4, rtol=1e-5)
    torch.testing.assert_close(part[1].double().sum(0), (g * xm).sum(0), atol=1e-5 * float((g * xm).abs().sum(0).max()) + 1e-4,
                               rtol=1e-5)
    # the node's finalize consumes it like the standalone reduction's partials
    ext = apex._native.require("conv").conv
    istd = torch.rand(c, device="cuda") + 0.5
    coef_b, gw, gb = ext.bnbwd_finalize(part, float(g.size(0)), mean, istd, None)
    torch.testing.assert_close(gb.double(), g.sum(0), atol=1e-3 * scale, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_gpu_tap_dgrad_prefetched_weight_images_bitwise(monkeypatch, stride):
    """APEX_AMD_TAP_PREFETCH (opt-in): the data-gradient weight images built on a side stream
    during the forward give the in-line dgrad bitwise, and a weight changed in place after the
    prefetch falls back to in-line images."""
    from apex.ops import conv as convops

    monkeypatch.setattr(convops, "_TAP_PREFETCH", True)
    torch.manual_seed(11 + stride)
    dt = torch.bfloat16
    n, c, k, h = 3, 128, 128, 14
    w = (torch.randn(k, c, 3, 3, device="cuda") * 0.05).to(dt).contiguous(memory_format=torch.channels_last)
    oh = (h + 2 - 3) // stride + 1
    gy = torch.randn(n, k, oh, oh, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    shape = (n, c, h, h)
    pre = convops.tap_images_async(w, shape, stride, 1)
    assert pre is not None
    want = convops.conv_tap_dgrad(gy, w, shape, stride, 1)
    got = convops.conv_tap_dgrad(gy, w, shape, stride, 1, pre=pre)
    assert torch.equal(got, want)
    pre = convops.tap_images_async(w, shape, stride, 1)
    with torch.no_grad():
        w.mul_(2)
    assert torch.equal(convops.conv_tap_dgrad(gy, w, shape, stride, 1, pre=pre),
                       convops.conv_tap_dgrad(gy, w, shape, stride, 1))


def test_tap_prefetch_is_off_on_cpu_tensors():
    from apex.ops import conv as convops

    w = torch.randn(64, 64, 3, 3).contiguous(memory_format=torch.channels_last)
    assert convops.tap_images_async(w, (1, 64, 8, 8), 1, 1) is None
