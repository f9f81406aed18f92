"""K-streamed fused 1x1 convolutions (csrc/conv/conv1x1_ks.hip): the deep reductions (k 1024 /
2048) of ResNet stages 3-4 through ``apex._C.conv.bn1x1`` / ``bn1x1_addrelu`` / ``dgrad_bnred``,
which route there when the resident-weight kernel cannot hold the weight tile.  Each against a
float64 torch reference of the same bf16 / fp16 operands; the operand prologues bitwise against
the standalone BN passes they replace (bn_nhwc apply / bwd_apply)."""
import pytest
import torch

# m, k, ncols: ragged row counts (m % 256 != 0), every column tile (256 / 128 / 64 chosen by the
# tile-count rule), both reductions of the ResNet-50 shapes
SHAPES = [
    (1000, 1024, 256),
    (777, 2048, 512),
    (3000, 1024, 128),
    (2100, 2048, 192),
    (513, 1024, 1024),
]


def _ext():
    import apex

    return apex._native.require("conv").conv


def _bn():
    import apex

    return apex._native.require("bn_nhwc").bn_nhwc


def _close(a, b, tol):
    scale = max(1.0, float(b.abs().max()))
    err = float((a.double() - b.double()).abs().max())
    assert err <= tol * scale, (err, scale)


def test_ks_shape_rule_cpu(monkeypatch):
    """The Python routing takes k 1024 / 2048 native only with the K-streamed kernel enabled
    (opt-in: APEX_AMD_C1KS=1)."""
    from apex.ops import bottleneck_bn as bb

    assert bb._k_native(512) and not bb._k_native(96)
    for on in (False, True):
        monkeypatch.setattr(bb, "_KS", on)
        assert bb._k_native(1024) == on and bb._k_native(2048) == on and bb._ks_only(1024) == on
        assert not bb._ks_only(512)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m,k,nc", SHAPES)
def test_gpu_ks_forward_and_stats(dtype, m, k, nc):
    ext = _ext()
    assert ext.ks1x1_supported(m, k, nc)
    torch.manual_seed(m + k + nc)
    a = torch.randn(m, k, device="cuda").to(dtype)
    w = (torch.randn(nc, k, device="cuda") * 0.03).to(dtype)
    shift = torch.randn(nc, device="cuda") * 0.1
    y, part, _ = ext.bn1x1(a, w, False, None, shift, True)
    ref = a.double() @ w.double().t()
    _close(y, ref, 1e-2)
    d = ref - shift.double()  # the epilogue sums the fp32 accumulators, before the output rounding
    assert part.shape[0] == 2 and part.shape[2] == nc
    torch.testing.assert_close(part[0].double().sum(0), d.sum(0), atol=1e-2 + 1e-4 * float(d.abs().sum(0).max()),
                               rtol=1e-3)
    torch.testing.assert_close(part[1].double().sum(0), (d * d).sum(0), rtol=2e-3, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,nc", SHAPES[:3])
@pytest.mark.parametrize("dual", [False, True])
def test_gpu_ks_addrelu_matches_apply_pass(m, k, nc, dual):
    """The deferred block output at stage 3-4 widths: bitwise the apply / dual-apply pass."""
    ext, bn = _ext(), _bn()
    torch.manual_seed(7 + m)
    dt = torch.bfloat16
    y3 = torch.randn(m, k, device="cuda").to(dt)
    res = torch.randn(m, k, device="cuda").to(dt)
    c3 = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3])
    cd = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3])
    w = (torch.randn(nc, k, device="cuda") * 0.03).to(dt)
    shift = torch.randn(nc, device="cuda") * 0.1
    if dual:
        want, want_bits = bn.apply(y3, res, c3, True, True, cd)
    else:
        want, want_bits = bn.apply(y3, res, c3, True, True)
    y, part, out, bits = ext.bn1x1_addrelu(y3, res, c3, w, shift, split=True, res_coef=cd if dual else None)
    assert torch.equal(out, want.view_as(out))
    assert torch.equal(bits.view(-1), want_bits.view(-1))
    ref = out.double() @ w.double().t()
    _close(y, ref, 1e-2)
    d = ref - shift.double()
    torch.testing.assert_close(part[0].double().sum(0), d.sum(0), atol=1e-2 + 1e-4 * float(d.abs().sum(0).max()),
                               rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("m,k,nc", SHAPES)
def test_gpu_ks_dgrad(dtype, m, k, nc):
    """dX = g . W with W [k, ncols] read k-major (transposed LDS reads)."""
    ext = _ext()
    torch.manual_seed(3 + m)
    g = torch.randn(m, k, device="cuda").to(dtype)
    wt = (torch.randn(k, nc, device="cuda") * 0.03).to(dtype)
    dx, _, _ = ext.bn1x1(g, wt, True, None, None, False)
    _close(dx, g.double() @ wt.double(), 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,nc", SHAPES[:4])
@pytest.mark.parametrize("red", [False, True])
def test_gpu_ks_dgrad_bn_prologue_and_reduction(m, k, nc, red):
    """conv3's data gradient at stages 3-4: bn3's dx on the operand load (written out bitwise the
    bwd_apply pass) and, with ``red``, bn2's ReLU mask recomputed from its input and its backward
    sums in the epilogue."""
    ext, bn = _ext(), _bn()
    torch.manual_seed(19 + m)
    dt = torch.bfloat16
    dm = torch.randn(m, k, device="cuda").to(dt)
    y3 = torch.randn(m, k, device="cuda").to(dt)
    wt = (torch.randn(k, nc, device="cuda") * 0.03).to(dt)
    cf = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3])
    cb = torch.cat([torch.randn(k, device="cuda"), torch.randn(k, device="cuda") * 0.1,
                    torch.randn(k, device="cuda") * 0.1])
    want_dx = bn.bwd_apply(dm, y3, cf, cb)
    if not red:
        dz, _, dx3 = ext.bn1x1(dm, wt, True, cb, None, False, None, y3, True)
        assert torch.equal(dx3, want_dx)
        _close(dz, want_dx.double() @ wt.double(), 1e-2)
        return
    y2 = torch.randn(m, nc, device="cuda").to(dt)
    c2 = torch.cat([torch.rand(nc, device="cuda") + 0.5, torch.randn(nc, device="cuda") * 0.3])
    mean2 = torch.randn(nc, device="cuda") * 0.1
    dz, part, dx3 = ext.dgrad_bnred(dm, wt, None, None, y2, mean2, coef=c2, py=y3, pcoef=cb, want_aout=True)
    assert torch.equal(dx3, want_dx)
    full = want_dx.double() @ wt.double()
    mask = (y2.float() * c2[:nc] + c2[nc:]) > 0
    # the kernel masks its own bf16-rounded result: compare against the rounded full product
    _close(dz, torch.where(mask, full, torch.zeros_like(full)), 1e-2)
    assert torch.equal(dz == 0, ~mask | (dz == 0))
    gq = dz.double()
    torch.testing.assert_close(part[0].double().sum(0), gq.sum(0), atol=1e-3 * float(gq.abs().sum(0).max()) + 1e-3,
                               rtol=1e-4)
    torch.testing.assert_close(part[1].double().sum(0), (gq * (y2.double() - mean2.double())).sum(0),
                               atol=1e-3 * float((gq * y2.double()).abs().sum(0).max()) + 1e-3, rtol=1e-4)
