"""BN-fused 1x1 convolution kernels (csrc/conv/conv1x1_bn.hip, ``apex._C.conv.bn1x1``):
y = pro(a) . W^T with the producing batch norm's apply + ReLU on the operand load, the consuming
batch norm's statistics partials in the epilogue, and the transposed-weight (data gradient) form —
each against the fp32 PyTorch composition of the same bf16/fp16 operands."""
import pytest
import torch

SHAPES = [
    # m, k, ncols
    (128, 64, 64),
    (1000, 64, 256),      # tail tile (m % 128 != 0)
    (4096, 256, 64),
    (2048, 256, 128),
    (3000, 128, 512),     # two 256-column groups
    (1536, 512, 128),
    (777, 128, 192),      # 64-column tile, odd row count
]


def _ext():
    import apex

    return apex._native.require("conv").conv


def _close(a, b, tol):
    scale = max(1.0, float(b.abs().max()))
    err = float((a.float() - b.float()).abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m,k,nc", SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_gpu_bn1x1_forward_and_stats(dtype, m, k, nc, pro):
    ext = _ext()
    torch.manual_seed(0)
    a = (torch.randn(m, k, device="cuda") * 2 + 0.5).to(dtype)
    w = (torch.randn(nc, k, device="cuda") * 0.1).to(dtype)
    pcoef = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3]) if pro else None
    shift = torch.randn(nc, device="cuda") * 0.1
    y, part, _ = ext.bn1x1(a, w, False, pcoef, shift, True)
    af = a.float()
    if pro:
        af = torch.relu(af * pcoef[:k] + pcoef[k:]).to(dtype).float()
    yr = af @ w.float().t()
    assert y.shape == (m, nc) and y.dtype == dtype
    _close(y, yr, 1e-2)
    # statistics: partials of the fp32 accumulators about `shift`, then the finalize
    rm = torch.zeros(nc, device="cuda")
    rv = torch.ones(nc, device="cuda")
    gam = torch.rand(nc, device="cuda") + 0.5
    bet = torch.randn(nc, device="cuda")
    sm, si, coef = ext.bn_finalize(part, float(m), shift, gam, bet, rm, rv, 1e-5, 0.1)
    mean, var = yr.mean(0), yr.var(0, unbiased=False)
    torch.testing.assert_close(sm, mean, atol=2e-3 * float(yr.std()), rtol=1e-3)
    torch.testing.assert_close(si, torch.rsqrt(var + 1e-5), atol=0, rtol=3e-3)
    torch.testing.assert_close(coef[:nc], gam * torch.rsqrt(var + 1e-5), atol=0, rtol=3e-3)
    torch.testing.assert_close(rm, 0.1 * mean, atol=2e-4 * float(yr.std()), rtol=1e-3)
    torch.testing.assert_close(rv, 0.9 + 0.1 * yr.var(0, unbiased=True), atol=0, rtol=3e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m,k,nc", SHAPES)
def test_gpu_bn1x1_dgrad_form(dtype, m, k, nc):
    """w_kmajor_out: y = a . W with W [k, ncols] (the data gradient of a [k-out, ncols-in] conv)."""
    ext = _ext()
    torch.manual_seed(1)
    a = torch.randn(m, k, device="cuda").to(dtype)
    w = (torch.randn(k, nc, device="cuda") * 0.1).to(dtype)
    y, part, _ = ext.bn1x1(a, w, True)
    assert part is None or part.numel() == 0
    _close(y, a.float() @ w.float(), 1e-2)
    res = torch.randn(m, nc, device="cuda").to(dtype)
    y2, _, _ = ext.bn1x1(a, w, True, None, None, False, res)
    _close(y2, a.float() @ w.float() + res.float(), 1e-2)


@pytest.mark.gpu
def test_gpu_bn1x1_large_mean_shift():
    """A channel mean far from zero: the running-mean shift keeps the variance accurate."""
    ext = _ext()
    torch.manual_seed(2)
    m, k, nc = 65536, 64, 64
    a = torch.randn(m, k, device="cuda").to(torch.bfloat16)
    w = (torch.randn(nc, k, device="cuda") * 0.02).to(torch.bfloat16)
    w[:, 0] = 1.0
    a[:, 0] = 300.0  # every output channel ~ 300 + small noise
    yr = a.float() @ w.float().t()
    shift = yr[:64].mean(0)  # a running-mean-like estimate
    _, part, _ = ext.bn1x1(a, w, False, None, shift, True)
    sm, si, _ = ext.bn_finalize(part, float(m), shift, None, None, None, None, 1e-5, 0.1)
    torch.testing.assert_close(si, torch.rsqrt(yr.var(0, unbiased=False) + 1e-5), atol=0, rtol=1e-2)


WGRAD_SHAPES = [
    # m, n (grad channels), k (activation channels)
    (1000, 256, 64),
    (4096, 64, 256),
    (2048, 128, 128),
    (3000, 512, 128),
    (1536, 128, 512),
    (640, 128, 64),
    (5000, 64, 128),
    (4000, 64, 64),
    (700, 192, 320),
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m,n,k", WGRAD_SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_gpu_wgrad1x1(dtype, m, n, k, pro):
    """dW = g^T . pro(x) against fp32 torch, pro = the producing BN's apply + ReLU."""
    ext = _ext()
    torch.manual_seed(3)
    g = torch.randn(m, n, device="cuda").to(dtype)
    x = (torch.randn(m, k, device="cuda") + 0.3).to(dtype)
    xcoef = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3]) if pro else None
    xf = x.float()
    if pro:
        xf = torch.relu(xf * xcoef[:k] + xcoef[k:]).to(dtype).float()
    ref = g.float().t() @ xf
    dw = ext.wgrad1x1(g, x, xcoef, torch.float32)
    assert dw.shape == (n, k)
    _close(dw, ref, 2e-3)
    dw16 = ext.wgrad1x1(g, x, xcoef)
    assert dw16.dtype == dtype
    _close(dw16, ref, 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m,k,nc", SHAPES)
def test_gpu_bn1x1_dgrad_bn_backward_prologue(dtype, m, k, nc):
    """dgrad form with the BN-backward prologue: a' = c0 * dm + c1 * y + c2 per reduction
    channel, the product a' . W, and a' itself written out (aout)."""
    ext = _ext()
    torch.manual_seed(4)
    dm = torch.randn(m, k, device="cuda").to(dtype)
    y = (torch.randn(m, k, device="cuda") + 0.2).to(dtype)
    w = (torch.randn(k, nc, device="cuda") * 0.1).to(dtype)
    cb = torch.randn(3 * k, device="cuda") * 0.5
    out, _, aout = ext.bn1x1(dm, w, True, cb, None, False, None, y, True)
    ap = (cb[:k] * dm.float() + cb[k:2 * k] * y.float() + cb[2 * k:]).to(dtype)
    _close(aout, ap, 1e-2)
    _close(out, ap.float() @ w.float(), 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,stride,h", [(64, 64, 1, 14), (128, 256, 2, 16), (256, 256, 1, 7)])
def test_gpu_tap_conv_bn_statistics_epilogue(cin, cout, stride, h):
    """3x3 implicit-GEMM forward with the consuming BN's statistics in the epilogue
    (ops.conv.conv_tap_forward(stats_shift=...)) -> finalize == torch batch mean / var."""
    import torch.nn.functional as F
    from apex.ops import conv as C

    ext = _ext()
    torch.manual_seed(5)
    x = (torch.randn(3, cin, h, h, device="cuda") + 0.3).to(torch.bfloat16).to(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).to(memory_format=torch.channels_last)
    shift = torch.randn(cout, device="cuda") * 0.1
    y, part = C.conv_tap_forward(x, w, stride, 1, stats_shift=shift)
    yr = F.conv2d(x.float(), w.float(), None, stride, 1)
    assert float((y.float() - yr).abs().max()) <= 1e-2 * max(1.0, float(yr.abs().max()))
    y2 = yr.permute(0, 2, 3, 1).reshape(-1, cout)
    sm, si, _ = ext.bn_finalize(part, float(y2.size(0)), shift, None, None, None, None, 1e-5, 0.1)
    torch.testing.assert_close(sm, y2.mean(0), atol=3e-3 * float(y2.std()), rtol=2e-3)
    torch.testing.assert_close(si, torch.rsqrt(y2.var(0, unbiased=False) + 1e-5), atol=0, rtol=5e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,nc", [(1000, 256, 64), (2048, 64, 256), (777, 512, 128)])
@pytest.mark.parametrize("mode", ["bits", "coef", "coef+pro"])
def test_gpu_dgrad_bnred(m, k, nc, mode):
    """dgrad form with the BN-backward reduction epilogue: out = mask(g' . W + res), partial
    sums of out and out * (x - mean); the mask from ReLU bits or recomputed from x and the BN's
    apply coefficients; optionally the BN-backward prologue g' = c0 g + c1 py + c2 (aout = g')."""
    ext = _ext()
    torch.manual_seed(6)
    dt = torch.bfloat16
    g = torch.randn(m, k, device="cuda").to(dt)
    w = (torch.randn(k, nc, device="cuda") * 0.1).to(dt)
    res = torch.randn(m, nc, device="cuda").to(dt)
    x = torch.randn(m, nc, device="cuda").to(dt)
    mean = torch.randn(nc, device="cuda") * 0.1
    coef = torch.cat([torch.rand(nc, device="cuda") + 0.5, torch.randn(nc, device="cuda") * 0.3])
    if mode == "bits":
        maskb = torch.rand(m, nc, device="cuda") > 0.4
        wts = (2 ** torch.arange(8, device="cuda")).view(1, 8)
        bits = (maskb.view(-1, 8).long() * wts).sum(1).to(torch.uint8)
        kw = dict(bits=bits)
    else:
        maskb = (x.float() * coef[:nc] + coef[nc:]) > 0
        kw = dict(bits=None, coef=coef)
    gp = g
    if mode == "coef+pro":
        py = torch.randn(m, k, device="cuda").to(dt)
        pc = torch.randn(3 * k, device="cuda") * 0.5
        gp = (pc[:k] * g.float() + pc[k:2 * k] * py.float() + pc[2 * k:]).to(dt)
        kw.update(py=py, pcoef=pc, want_aout=True)
    out, part, aout = ext.dgrad_bnred(g, w, res, kw.pop("bits"), x, mean, **kw)
    ref = torch.where(maskb, (gp.float() @ w.float() + res.float()).to(dt).float(), torch.zeros(()).cuda())
    _close(out, ref, 2e-2)
    if mode == "coef+pro":
        _close(aout, gp, 1e-2)
    s1 = part[0].sum(0)
    s2 = part[1].sum(0)
    of = out.float()
    torch.testing.assert_close(s1, of.sum(0), atol=0.05 * float(of.abs().sum(0).max()) / 100 + 0.5, rtol=2e-2)
    torch.testing.assert_close(s2, (of * (x.float() - mean)).sum(0), atol=1.0, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,stride,h,batch", [(64, 64, 1, 14, 3), (128, 128, 2, 16, 2), (64, 128, 1, 9, 2),
                                                     (256, 256, 2, 14, 2), (128, 192, 1, 7, 5)])
@pytest.mark.parametrize("pro", [False, True])
def test_gpu_wgrad3x3_gather(cin, cout, stride, h, batch, pro):
    """3x3 weight gradient on the split-M kernel with the per-tap input gather (zero padding) and
    the optional BN-apply + ReLU prologue, against fp32 torch's convolution weight gradient."""
    ext = _ext()
    torch.manual_seed(7)
    dt = torch.bfloat16
    x = (torch.randn(batch, cin, h, h, device="cuda") + 0.2).to(dt).to(memory_format=torch.channels_last)
    oh = (h + 2 - 3) // stride + 1
    gy = torch.randn(batch, cout, oh, oh, device="cuda").to(dt).to(memory_format=torch.channels_last)
    xcoef = torch.cat([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.3]) if pro else None
    xf = x.float()
    if pro:
        xf = torch.relu(xf * xcoef[:cin].view(1, -1, 1, 1) + xcoef[cin:].view(1, -1, 1, 1)).to(dt).float()
    w = torch.zeros(cout, cin, 3, 3, device="cuda")
    ref = torch.ops.aten.convolution_backward(gy.float(), xf, w, None, [stride, stride], [1, 1], [1, 1], False,
                                              [0, 0], 1, [False, True, False])[1]
    dw = ext.wgrad3x3(gy.permute(0, 2, 3, 1), x.permute(0, 2, 3, 1), stride, xcoef, torch.float32)
    assert dw.shape == ref.shape
    _close(dw, ref, 2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,ncols", [(777, 256, 64), (1000, 512, 128), (300, 256, 128), (64, 64, 64)])
@pytest.mark.parametrize("dual", [False, True])
def test_gpu_bn1x1_addrelu_matches_apply_pass(m, k, ncols, dual):
    """The deferred block output (conv1x1_bn kProBnAddRelu: the block below's output BN + shortcut
    + ReLU computed on the conv's operand load, written out with its ReLU bits) is BITWISE the
    output and bit mask of the standalone apply / dual-apply pass it replaces, and the conv output
    and its statistics match fp32 torch on that operand."""
    import apex
    from apex import _native

    bn = _native.require("bn_nhwc").bn_nhwc
    ext = _ext()
    torch.manual_seed(m + k)
    dt = torch.bfloat16
    y3 = torch.randn(m, k, device="cuda").to(dt)
    res = torch.randn(m, k, device="cuda").to(dt)
    c3 = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3])
    cd = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3])
    w = (torch.randn(ncols, k, device="cuda") * 0.05).to(dt)
    shift = torch.randn(ncols, device="cuda") * 0.1
    if dual:
        want, want_bits = bn.apply(y3, res, c3, True, True, cd)
        pc = torch.cat([c3[:k], cd[:k], c3[k:], cd[k:]])
    else:
        want, want_bits = bn.apply(y3, res, c3, True, True)
        pc = torch.cat([c3[:k], torch.ones(k, device="cuda"), c3[k:], torch.zeros(k, device="cuda")])
    y, part, out, bits = ext.bn1x1_addrelu(y3, res, pc, w, shift)
    assert torch.equal(out, want.view_as(out))
    assert torch.equal(bits.view(-1), want_bits.view(-1))
    # the split-coefficient form (bn3's [2K] and the downsample BN's [2K] or None, assembled on the
    # kernel's LDS load) is bitwise the concatenated one
    y_s, part_s, out_s, bits_s = ext.bn1x1_addrelu(y3, res, c3, w, shift, split=True, res_coef=cd if dual else None)
    assert torch.equal(out_s, out) and torch.equal(bits_s, bits) and torch.equal(y_s, y)
    assert torch.equal(part_s, part)
    ref = out.float() @ w.float().t()
    _close(y, ref, 1e-2)
    d = y.float() - shift
    torch.testing.assert_close(part[0].sum(0), d.sum(0), atol=0.05 + 1e-3 * float(d.abs().sum(0).max()), rtol=1e-3)


def _scatter_sub(sub, n, h, w):
    """[N * ceil(h/2) * ceil(w/2), C] stride-2 subsample gradient -> dense [N * h * w, C] (zeros at odd y / x)."""
    c = sub.size(1)
    dense = torch.zeros(n, h, w, c, device=sub.device, dtype=torch.float32)
    dense[:, ::2, ::2] = sub.float().view(n, (h + 1) // 2, (w + 1) // 2, c)
    return dense.view(-1, c)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,k,nc", [(2, 56, 56, 64, 256), (3, 28, 28, 128, 512), (2, 7, 9, 256, 128)])
@pytest.mark.parametrize("red", [False, True])
def test_gpu_dgrad_subsampled_residual(n, h, w, k, nc, red):
    """The strided 1x1 downsample's data gradient [N, ceil(h/2), ceil(w/2), C] added at even (y, x)
    in the dgrad epilogue (conv1x1_bn.hip rs_*): plain dgrad form and the BN-reduction form."""
    ext = _ext()
    torch.manual_seed(11)
    dt = torch.bfloat16
    m = n * h * w
    g = torch.randn(m, k, device="cuda").to(dt)
    wt = (torch.randn(k, nc, device="cuda") * 0.1).to(dt)
    sub = torch.randn(n * ((h + 1) // 2) * ((w + 1) // 2), nc, device="cuda").to(dt)
    dense = _scatter_sub(sub, n, h, w)
    if not red:
        out = ext.bn1x1(g, wt, True, None, None, False, sub, res_h=h, res_w=w)[0]
        ref = (g.float() @ wt.float() + dense).to(dt)
        _close(out, ref, 2e-2)
        # the dense-residual path agrees with it
        out_d = ext.bn1x1(g, wt, True, None, None, False, dense.to(dt))[0]
        _close(out, out_d, 1e-2)
        return
    x = torch.randn(m, nc, device="cuda").to(dt)
    mean = torch.randn(nc, device="cuda") * 0.1
    maskb = torch.rand(m, nc, device="cuda") > 0.4
    wts = (2 ** torch.arange(8, device="cuda")).view(1, 8)
    bits = (maskb.view(-1, 8).long() * wts).sum(1).to(torch.uint8)
    out, part, _ = ext.dgrad_bnred(g, wt, sub, bits, x, mean, res_h=h, res_w=w)
    out_d, part_d, _ = ext.dgrad_bnred(g, wt, dense.to(dt), bits, x, mean)
    ref = torch.where(maskb, (g.float() @ wt.float() + dense).to(dt).float(), torch.zeros(()).cuda())
    _close(out, ref, 2e-2)
    torch.testing.assert_close(out, out_d)
    torch.testing.assert_close(part, part_d)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,c", [(2, 56, 56, 256), (3, 7, 9, 64), (1, 28, 28, 1024)])
def test_gpu_subsample2x(n, h, w, c):
    """The stride-2 1x1 operand: y[n][i][j] = x[n][2i][2j], dense NHWC rows (csrc/conv/layout.hip)."""
    ext = _ext()
    x = torch.randn(n * h * w, c, device="cuda").to(torch.bfloat16)
    y = ext.subsample2x(x, n, h, w)
    assert torch.equal(y, x.view(n, h, w, c)[:, ::2, ::2].reshape(-1, c))


@pytest.mark.gpu
@pytest.mark.parametrize("k,c,ks,taps", [(64, 64, 3, list(range(9))), (128, 256, 3, list(range(9))),
                                         (72, 40, 3, [0, 2, 6, 8]), (512, 512, 3, [4]), (256, 1024, 1, [0]),
                                         (200, 136, 3, [1, 7])])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gpu_tap_weights(k, c, ks, taps, dt):
    """The data-gradient weight image dst[c][j][k] = w[k][taps[j]][c] (csrc/conv/layout.hip): bitwise
    the permute + stack copy it replaces in ops/conv.py conv_tap_dgrad, ragged tiles included."""
    ext = _ext()
    w = torch.randn(k, c, ks, ks, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    out = ext.tap_weights(w, taps)
    wk = w.permute(1, 2, 3, 0)
    ref = torch.stack([wk[:, t // ks, t % ks, :] for t in taps], 1).contiguous()
    assert out.shape == (c, len(taps), k) and torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,nc,linked", [(4096, 64, 256, False), (4096, 64, 256, True), (2048, 128, 512, True),
                                           (1024, 512, 1024, False), (1024, 512, 1024, True),
                                           (1000, 256, 1024, True)])
def test_gpu_bn_dx_prologue_with_recomputed_mask(m, k, nc, linked):
    """bn1's dx as the conv1 dgrad operand prologue with the ReLU mask recomputed from y1
    (kProBnBwdMask, pcoef [5k] from bn_nhwc.bwd_coef): the written a' is bitwise the standalone
    reduction + dx passes' dx, and the dgrad (plain and with the block-below reduction) bitwise the
    dgrad of that dx."""
    from apex import _native

    ext = _ext()
    bn = _native.require("bn_nhwc").bn_nhwc
    torch.manual_seed(5)
    dt = torch.bfloat16
    y1 = torch.randn(m, k, device="cuda").to(dt)
    dz = torch.randn(m, k, device="cuda").to(dt)
    wt = (torch.randn(k, nc, device="cuda") * 0.1).to(dt)
    g1 = torch.rand(k, device="cuda") + 0.5
    b1 = torch.randn(k, device="cuda") * 0.1
    rm, rv = torch.zeros(k, device="cuda"), torch.ones(k, device="cuda")
    sm, si, c1 = bn.stats(y1, g1, b1, rm, rv, 0.1, 1e-5)
    c1 = c1.view(-1)
    ref_dx, _, ref_gw, ref_gb = bn.bwd(dz, y1, None, g1, sm, si, c1, True, False)
    pc5, gw, gb = bn.bwd_coef(dz, y1, g1, sm, si, c1)
    assert torch.equal(gw, ref_gw) and torch.equal(gb, ref_gb)
    short = torch.randn(m, nc, device="cuda").to(dt)
    if not linked:
        out, _, aout = ext.bn1x1(dz, wt, True, pc5.view(-1), None, False, short, y1, True)
        ref_out = ext.bn1x1(ref_dx, wt, True, None, None, False, short)[0]
        assert torch.equal(aout, ref_dx)
        assert torch.equal(out, ref_out)
        return
    x = torch.randn(m, nc, device="cuda").to(dt)
    mean = torch.randn(nc, device="cuda") * 0.1
    bits = torch.randint(0, 256, (m * nc // 8,), device="cuda", dtype=torch.uint8)
    out, part, aout = ext.dgrad_bnred(dz, wt, short, bits, x, mean, py=y1, pcoef=pc5.view(-1), want_aout=True)
    ref_out, ref_part, _ = ext.dgrad_bnred(ref_dx, wt, short, bits, x, mean)
    assert torch.equal(aout, ref_dx)
    assert torch.equal(out, ref_out)
    torch.testing.assert_close(part.sum(1), ref_part.sum(1), rtol=1e-5, atol=1e-3)
