"""FusedLayerNorm / MixedFusedLayerNorm / FusedRMSNorm numerics.

Model: reference tests/L0/run_fused_layer_norm/test_fused_layer_norm.py:10-111 (fused module vs
``F.layer_norm`` in fp32 / half / bf16).  GPU tests compare the gfx950 kernels against a plain
fp32 PyTorch reference of the same op, over widths that exercise every register-resident
geometry (norm_common.h pick_cfg; 16-wave wide rows up to 65536) and the generic path (n2 % 8 != 0,
n2 > 65536, fp32 rows past 32768 in the backward)."""
import pytest
import torch
import torch.nn.functional as F

from apex.normalization import FusedLayerNorm, MixedFusedLayerNorm

try:
    from apex.normalization import FusedRMSNorm, MixedFusedRMSNorm
except ImportError:  # pragma: no cover
    FusedRMSNorm = MixedFusedRMSNorm = None


def _ref_ln(x, w, b, eps, rms=False):
    xf = x.float()
    if rms:
        y = xf * torch.rsqrt((xf * xf).mean(-1, keepdim=True) + eps)
    else:
        y = (xf - xf.mean(-1, keepdim=True)) * torch.rsqrt(xf.var(-1, unbiased=False, keepdim=True) + eps)
    if w is not None:
        y = y * w.float()
    if b is not None:
        y = y + b.float()
    return y


def test_cpu_module_matches_functional():
    torch.manual_seed(0)
    m = FusedLayerNorm(32)
    x = torch.randn(4, 7, 32, requires_grad=True)
    y = m(x)
    yr = F.layer_norm(x, (32,), m.weight, m.bias, m.eps)
    torch.testing.assert_close(y, yr)
    y.sum().backward()


def test_cpu_mixed_dtype_output():
    m = MixedFusedLayerNorm(16).to(torch.bfloat16)
    x = torch.randn(3, 16)
    assert m(x).dtype in (torch.bfloat16, torch.float32)


@pytest.mark.skipif(FusedRMSNorm is None, reason="no RMSNorm")
def test_cpu_rms_norm():
    torch.manual_seed(0)
    m = FusedRMSNorm(24)
    x = torch.randn(5, 24, requires_grad=True)
    y = m(x)
    torch.testing.assert_close(y, _ref_ln(x, m.weight, None, m.eps, rms=True))
    y.sum().backward()


# 20008: generic (n2 % 8 != 0); 24576 .. 65536: the 16-wave wide kernels (40000: a partial last
# vector column block; fp32 at 65536 takes the generic backward)
WIDTHS = [64, 768, 1000, 1024, 2048, 3072, 4096, 5120, 8192, 12288, 16384, 20008, 24576, 32768, 40000, 65536]
TOL = {torch.float32: (1e-4, 1e-4), torch.float16: (2e-2, 1e-2), torch.bfloat16: (5e-2, 2e-2)}


@pytest.mark.gpu
@pytest.mark.parametrize("n2", WIDTHS)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("affine", [True, False])
def test_gpu_layer_norm(n2, dtype, affine):
    import apex

    assert apex._native.available()
    torch.manual_seed(n2)
    n1 = 67  # not a multiple of the rows-per-block
    x = (torch.randn(n1, n2, device="cuda") * 3 + 1).to(dtype).requires_grad_(True)
    m = FusedLayerNorm(n2, elementwise_affine=affine).cuda().to(dtype)
    if affine:
        with torch.no_grad():
            m.weight.copy_(torch.rand(n2) + 0.5)
            m.bias.copy_(torch.randn(n2) * 0.1)
    y = m(x)
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().float().requires_grad_(True) if affine else None
    br = m.bias.detach().float().requires_grad_(True) if affine else None
    yr = _ref_ln(xr, wr, br, m.eps)
    atol, rtol = TOL[dtype]
    torch.testing.assert_close(y.float(), yr, atol=atol, rtol=rtol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=atol * 4, rtol=rtol * 4)
    if affine:
        scale = max(1.0, float(wr.grad.abs().max()))
        torch.testing.assert_close(m.weight.grad.float() / scale, wr.grad / scale, atol=atol * 4, rtol=rtol * 4)
        scale = max(1.0, float(br.grad.abs().max()))
        torch.testing.assert_close(m.bias.grad.float() / scale, br.grad / scale, atol=atol * 4, rtol=rtol * 4)


@pytest.mark.gpu
@pytest.mark.parametrize("n2", [1024, 4096, 1000])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gpu_mixed_dtypes(n2, dtype):
    """MixedFusedLayerNorm: low-precision input, fp32 gamma/beta, output in weight dtype."""
    torch.manual_seed(1)
    x = torch.randn(33, n2, device="cuda", dtype=dtype, requires_grad=True)
    m = MixedFusedLayerNorm(n2).cuda()
    y = m(x)
    assert y.dtype == m.weight.dtype
    xr = x.detach().float().requires_grad_(True)
    yr = _ref_ln(xr, m.weight.detach(), m.bias.detach(), m.eps)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=1e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=5e-2)


@pytest.mark.gpu
@pytest.mark.skipif(FusedRMSNorm is None, reason="no RMSNorm")
@pytest.mark.parametrize("n2", [512, 2048, 8192, 1000, 49152])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gpu_rms_norm(n2, dtype):
    torch.manual_seed(2)
    x = torch.randn(40, n2, device="cuda", dtype=dtype, requires_grad=True)
    m = FusedRMSNorm(n2).cuda().to(dtype)
    with torch.no_grad():
        m.weight.copy_(torch.rand(n2) + 0.5)
    y = m(x)
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().float().requires_grad_(True)
    yr = _ref_ln(xr, wr, None, m.eps, rms=True)
    atol, rtol = TOL[dtype]
    torch.testing.assert_close(y.float(), yr, atol=atol, rtol=rtol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=atol * 4, rtol=rtol * 4)
    scale = max(1.0, float(wr.grad.abs().max()))
    torch.testing.assert_close(m.weight.grad.float() / scale, wr.grad / scale, atol=atol * 4, rtol=rtol * 4)


@pytest.mark.gpu
def test_gpu_layer_norm_deterministic():
    torch.manual_seed(3)
    x = torch.randn(4096, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    m = FusedLayerNorm(1024).cuda().to(torch.bfloat16)
    g = torch.randn_like(x)
    outs = []
    for _ in range(2):
        x.grad = None
        m.zero_grad()
        m(x).backward(g)
        outs.append((x.grad.clone(), m.weight.grad.clone(), m.bias.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_cpu_fast_layer_norm_module():
    from apex.contrib.layer_norm import FastLayerNorm

    torch.manual_seed(0)
    m = FastLayerNorm(48)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    x = torch.randn(6, 5, 48, requires_grad=True)
    ref = torch.nn.functional.layer_norm(x, (48,), m.weight, m.bias, 1e-5)
    y = m(x)
    torch.testing.assert_close(y, ref, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, m.weight, m.bias), g)
    exp = torch.autograd.grad(ref, (x, m.weight, m.bias), g)
    for a, b in zip(got, exp):
        torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("hidden", [768, 1024, 4096, 12288, 25600, 32768, 65536])
@pytest.mark.parametrize("itype,wtype", [(torch.bfloat16, torch.bfloat16), (torch.float16, torch.float32),
                                         (torch.float32, torch.float32)])
def test_gpu_fast_layer_norm(hidden, itype, wtype):
    """reference apex/contrib/test/layer_norm/test_fast_layer_norm.py: hidden sizes x dtype combos."""
    from apex.contrib.layer_norm import FastLayerNorm

    torch.manual_seed(hidden)
    m = FastLayerNorm(hidden).cuda().to(wtype)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    x = torch.randn(64, hidden, device="cuda").to(itype).requires_grad_(True)
    y = m(x)
    assert y.dtype == itype
    xr = x.detach().float().requires_grad_(True)
    wr, br = m.weight.detach().float().requires_grad_(True), m.bias.detach().float().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xr, (hidden,), wr, br, 1e-5)
    tol = 2e-2 if itype != torch.float32 else 1e-4
    torch.testing.assert_close(y.float(), ref, atol=tol, rtol=tol)
    g = torch.randn_like(ref)
    y.backward(g.to(itype))
    ref.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)
    s = float(wr.grad.abs().max())
    torch.testing.assert_close(m.weight.grad.float() / s, wr.grad / s, atol=tol, rtol=tol)
    s = float(br.grad.abs().max())
    torch.testing.assert_close(m.bias.grad.float() / s, br.grad / s, atol=tol, rtol=tol)

@pytest.mark.gpu
@pytest.mark.parametrize("hidden", [1024, 768, 4096])
def test_gpu_layer_norm_with_residual_matches_autograd_sum(hidden):
    """(LN(x), x) as one node (the LayerNorm backward kernel adds the residual branch's gradient
    into dx) against the plain module + autograd's sum of the two branches."""
    from apex.normalization import FusedLayerNorm
    from apex.normalization.fused_layer_norm import layer_norm_with_residual

    torch.manual_seed(hidden)
    dt = torch.bfloat16
    ln = FusedLayerNorm(hidden).cuda().to(dt)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    x = torch.randn(3, 257, hidden, device="cuda").to(dt)
    gy = torch.randn_like(x)
    gr = torch.randn_like(x)
    xa = x.clone().requires_grad_(True)
    y, r = layer_norm_with_residual(ln, xa)
    torch.autograd.backward([y, r * 1.0], [gy, gr])
    ga, gwa, gba = xa.grad, ln.weight.grad.clone(), ln.bias.grad.clone()
    ln.weight.grad = ln.bias.grad = None
    xb = x.clone().requires_grad_(True)
    yb = ln(xb)
    torch.autograd.backward([yb, xb * 1.0], [gy, gr])
    assert torch.equal(y, yb)
    torch.testing.assert_close(ga.float(), xb.grad.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(gwa.float(), ln.weight.grad.float(), atol=0, rtol=0)
    torch.testing.assert_close(gba.float(), ln.bias.grad.float(), atol=0, rtol=0)


def test_layer_norm_with_residual_cpu_fallback():
    """Off the GPU the pair is the plain module output and the input itself; gradients sum."""
    from apex.normalization.fused_layer_norm import layer_norm_with_residual

    torch.manual_seed(0)
    ln = FusedLayerNorm(16)
    x = torch.randn(4, 16, requires_grad=True)
    y, r = layer_norm_with_residual(ln, x)
    assert r is x
    (y.sum() + (2 * r).sum()).backward()
    x2 = x.detach().clone().requires_grad_(True)
    (ln(x2).sum() + (2 * x2).sum()).backward()
    torch.testing.assert_close(x.grad, x2.grad)
