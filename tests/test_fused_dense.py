"""Fused dense / MLP / MFMA GEMM numerics.

Model: reference apex/contrib/test/fused_dense/test_fused_dense.py (y, dx, dw, db vs matmul) and
tests/L0/run_mlp/test_mlp.py (MLP vs nn.Sequential(Linear, ReLU, ...)).  GPU tests compare the
gfx950 MFMA kernel (all four operand-major combinations, every epilogue, ragged shapes) against
fp32 torch math."""
import pytest
import torch

from apex.fused_dense import FusedDense, FusedDenseGeluDense
from apex.mlp import MLP


def test_cpu_fused_dense_and_mlp():
    torch.manual_seed(0)
    m = FusedDense(16, 24)
    x = torch.randn(5, 16, requires_grad=True)
    y = m(x)
    torch.testing.assert_close(y, x @ m.weight.t() + m.bias)
    y.sum().backward()
    torch.testing.assert_close(m.bias.grad, torch.full((24,), 5.0))
    g = FusedDenseGeluDense(16, 32, 8)
    out = g(x)
    ref = torch.nn.functional.gelu(x @ g.weight1.t() + g.bias1, approximate="tanh") @ g.weight2.t() + g.bias2
    torch.testing.assert_close(out, ref)
    out.sum().backward()
    mlp = MLP([16, 32, 8])
    mlp(x).mean().backward()


def _ref_mm(a, a_kmajor, b, b_kmajor, m, n, k):
    A = a.float().view(m, k) if a_kmajor else a.float().view(k, m).t()
    B = b.float().view(n, k).t() if b_kmajor else b.float().view(k, n)
    return A @ B


SHAPES = [(128, 128, 64), (256, 384, 512), (200, 136, 72), (1000, 1032, 2048), (64, 4096, 1024), (3072, 1024, 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", SHAPES)
@pytest.mark.parametrize("a_kmajor,b_kmajor", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_gemm_layouts(m, n, k, a_kmajor, b_kmajor, dtype):
    import apex

    g = apex._native.require("gemm").gemm
    torch.manual_seed(m + n + k)
    a = torch.randn(m * k, device="cuda").to(dtype)
    b = torch.randn(k * n, device="cuda").to(dtype)
    if not a_kmajor and m % 8:
        pytest.skip("m-major A needs M % 8 == 0")
    c, _ = g.matmul(a, a_kmajor, b, b_kmajor, m, n, k)
    ref = _ref_mm(a, a_kmajor, b, b_kmajor, m, n, k)
    scale = (k ** 0.5)
    torch.testing.assert_close(c.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_gemm_epilogues(dtype):
    import apex

    g = apex._native.require("gemm").gemm
    torch.manual_seed(1)
    m, n, k = 300, 264, 320
    x = (torch.randn(m, k, device="cuda") * 0.3).to(dtype)
    w = (torch.randn(n, k, device="cuda") * 0.1).to(dtype)
    b = torch.randn(n, device="cuda").to(dtype)
    z = x.float() @ w.float().t() + b.float()
    tol = dict(atol=3e-2, rtol=3e-2)
    y, aux = g.linear(x, w, b, g.EPI_GELU, True)
    torch.testing.assert_close(aux.float(), z, **tol)
    torch.testing.assert_close(y.float(), torch.nn.functional.gelu(z, approximate="tanh"), **tol)
    y, _ = g.linear(x, w, b, g.EPI_RELU, False)
    torch.testing.assert_close(y.float(), torch.relu(z), **tol)
    y, _ = g.linear(x, w, b, g.EPI_SIGMOID, False)
    torch.testing.assert_close(y.float(), torch.sigmoid(z), **tol)
    dy = torch.randn(m, n, device="cuda").to(dtype)
    zz = z.to(dtype)
    dx = g.linear_dgrad(dy, w, g.EPI_NONE, None)
    torch.testing.assert_close(dx.float(), dy.float() @ w.float(), **tol)
    # activation-derivative epilogues (aux has the shape of the GEMM output: [m, k])
    auxk = torch.randn(m, k, device="cuda").to(dtype)
    base = dy.float() @ w.float()
    zt = auxk.float().requires_grad_(True)
    dg = torch.autograd.grad(torch.nn.functional.gelu(zt, approximate="tanh").sum(), zt)[0]
    torch.testing.assert_close(g.linear_dgrad(dy, w, g.EPI_DGELU, auxk).float(), base * dg, **tol)
    torch.testing.assert_close(g.linear_dgrad(dy, w, g.EPI_DRELU, auxk).float(), base * (auxk.float() > 0), **tol)
    s = torch.sigmoid(auxk.float()).to(dtype)
    torch.testing.assert_close(g.linear_dgrad(dy, w, g.EPI_DSIGMOID, s).float(),
                               base * s.float() * (1 - s.float()), **tol)
    dw = g.linear_wgrad(dy, x)
    torch.testing.assert_close(dw.float() / 10, (dy.float().t() @ x.float()) / 10, **tol)
    cs = g.column_sum(dy, torch.float32)
    torch.testing.assert_close(cs, dy.float().sum(0), atol=1e-2, rtol=1e-3)
    del zz


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["native", "lt", "lt_bgradb", "library", "auto"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gpu_fused_dense_reference_test(dtype, route, monkeypatch):
    """The reference's test shapes: 3 x 512 tokens, 1024 -> 3072 (dx, dw, db all checked), on the
    native kernels and under the measured per-shape routing."""
    from apex.fused_dense import fused_dense as fd

    if route == "lt_bgradb":
        route = "lt"
        monkeypatch.setenv("APEX_AMD_LT_BGRADB", "1")
    monkeypatch.setenv("APEX_AMD_DENSE_ROUTE", route)
    torch.manual_seed(0)
    x = torch.randn(3 * 512, 1024, device="cuda").to(dtype).requires_grad_(True)
    dense = FusedDense(1024, 3072).cuda().to(dtype)
    y = dense(x)
    xr = x.detach().float().requires_grad_(True)
    yr = xr @ dense.weight.float().t() + dense.bias.float()
    torch.testing.assert_close(y.float() / 8, yr / 8, atol=2e-2, rtol=2e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    dw_ref = dy.float().t() @ xr.detach()
    dx_ref = dy.float() @ dense.weight.float()
    db_ref = dy.float().sum(0)
    torch.testing.assert_close(x.grad.float() / 8, dx_ref / 8, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(dense.weight.grad.float() / 40, dw_ref / 40, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(dense.bias.grad.float() / 40, db_ref / 40, atol=2e-2, rtol=2e-2)
    if route == "auto":
        keys = [k for k in fd.route_table() if k[0] in ("dense_fwd", "dense_bwd") and k[1:4] == (1536, 3072, 1024)]
        assert len(keys) >= 2  # forward and backward were both timed and decided


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["native", "lt", "lt_bgradb", "lt_dgelu_pass", "library", "auto"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gpu_fused_dense_gelu_dense(dtype, route, monkeypatch):
    if route == "lt_bgradb":
        route = "lt"
        monkeypatch.setenv("APEX_AMD_LT_BGRADB", "1")
    if route == "lt_dgelu_pass":  # library dgrad + the one-pass dGeLU / column sum (A/B arm)
        import importlib

        route = "lt"
        monkeypatch.setattr(importlib.import_module("apex.fused_dense.fused_dense"), "_DGELU_ROUTE", "pass")
    monkeypatch.setenv("APEX_AMD_DENSE_ROUTE", route)
    torch.manual_seed(2)
    x = (torch.randn(2, 256, 512, device="cuda") * 0.5).to(dtype).requires_grad_(True)
    mod = FusedDenseGeluDense(512, 2048, 512).cuda().to(dtype)
    y = mod(x)
    xr = x.detach().float().requires_grad_(True)
    w1, b1, w2, b2 = [p.detach().float().requires_grad_(True) for p in (mod.weight1, mod.bias1, mod.weight2, mod.bias2)]
    yr = torch.nn.functional.gelu(xr @ w1.t() + b1, approximate="tanh") @ w2.t() + b2
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    dy = torch.randn_like(yr)
    y.backward(dy.to(dtype))
    yr.backward(dy)
    for got, ref in ((x.grad, xr.grad), (mod.weight1.grad, w1.grad), (mod.bias1.grad, b1.grad),
                     (mod.weight2.grad, w2.grad), (mod.bias2.grad, b2.grad)):
        s = max(1.0, float(ref.abs().max()))
        torch.testing.assert_close(got.float() / s, ref / s, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["native", "lt", "library"])
def test_gpu_fused_dense_fp32(route, monkeypatch):
    """fp32 GPU tensors take the torch ops on every route: the hipBLASLt wrapper only takes fp16 /
    bf16 operands of one dtype and must not be called with fp32 ones."""
    monkeypatch.setenv("APEX_AMD_DENSE_ROUTE", route)
    torch.manual_seed(3)
    x = torch.randn(64, 128, device="cuda", requires_grad=True)
    dense = FusedDense(128, 96).cuda()
    y = dense(x)
    y.backward(torch.ones_like(y))
    torch.testing.assert_close(y, x.detach() @ dense.weight.t() + dense.bias, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dense.bias.grad, torch.full((96,), 64.0, device="cuda"))
    mod = FusedDenseGeluDense(128, 256, 64).cuda()
    x2 = torch.randn(2, 32, 128, device="cuda", requires_grad=True)
    out = mod(x2)
    ref = torch.nn.functional.gelu(x2.detach() @ mod.weight1.t() + mod.bias1, approximate="tanh") @ mod.weight2.t()
    torch.testing.assert_close(out, ref + mod.bias2, atol=1e-4, rtol=1e-4)
    out.sum().backward()
    assert x2.grad is not None and torch.isfinite(x2.grad).all() and mod.bias1.grad is not None


@pytest.mark.gpu
@pytest.mark.parametrize("activation", ["none", "relu", "sigmoid"])
@pytest.mark.parametrize("bias", [True, False])
def test_gpu_mlp_vs_sequential(activation, bias):
    torch.manual_seed(3)
    sizes = [480, 1024, 1024, 512, 256]
    mlp = MLP(sizes, bias=bias, activation=activation).cuda().to(torch.bfloat16)
    layers = []
    for i in range(mlp.num_layers):
        lin = torch.nn.Linear(sizes[i], sizes[i + 1], bias=bias).cuda()
        with torch.no_grad():
            lin.weight.copy_(mlp.weights[i].float())
            if bias:
                lin.bias.copy_(mlp.biases[i].float())
        layers.append(lin)
        if activation == "relu":
            layers.append(torch.nn.ReLU())
        elif activation == "sigmoid":
            layers.append(torch.nn.Sigmoid())
    ref = torch.nn.Sequential(*layers)
    x = torch.rand(128, sizes[0], device="cuda") * 2 - 1
    xt = x.to(torch.bfloat16).requires_grad_(True)
    xr = xt.detach().float().requires_grad_(True)
    out = mlp(xt)
    out_ref = ref(xr)
    torch.testing.assert_close(out.float(), out_ref, atol=3e-2, rtol=3e-2)
    out.float().mean().mul(10.0).backward()
    out_ref.mean().mul(10.0).backward()
    s = max(1e-3, float(xr.grad.abs().max()))
    if activation == "relu":
        # bf16 pre-activations within rounding of 0 may flip the ReLU mask vs fp32: allow a
        # handful of such elements, everything else must match
        bad = ((xt.grad.float() / s - xr.grad / s).abs() > 3e-2 + 3e-2 * (xr.grad / s).abs()).float().mean()
        assert float(bad) < 1e-3, float(bad)
    else:
        torch.testing.assert_close(xt.grad.float() / s, xr.grad / s, atol=3e-2, rtol=3e-2)
    if bias:
        s = max(1e-3, float(ref[0].bias.grad.abs().max()))
        torch.testing.assert_close(mlp.biases[0].grad.float() / s, ref[0].bias.grad / s, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["force", "off"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (300, 520, 128), (1024, 768, 1024), (77, 4104, 192)])
def test_gpu_gemm256_nt_path(mode, m, n, k, monkeypatch):
    """The 256x256 LDS-DMA kernel (forced on small shapes) and the 128x128 kernel agree with fp32
    math on the forward-linear (NT) layout, with ragged M / N edges and every epilogue."""
    import apex

    monkeypatch.setenv("APEX_AMD_GEMM256", mode)
    g = apex._native.require("gemm").gemm
    torch.manual_seed(m + n)
    x = (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda") * 0.2).to(torch.bfloat16)
    b = torch.randn(n, device="cuda").to(torch.bfloat16)
    z = x.float() @ w.float().t() + b.float()
    tol = dict(atol=3e-2, rtol=3e-2)
    y, _ = g.linear(x, w, b, g.EPI_NONE, False)
    torch.testing.assert_close(y.float(), z, **tol)
    y, aux = g.linear(x, w, b, g.EPI_GELU, True)
    torch.testing.assert_close(aux.float(), z, **tol)
    torch.testing.assert_close(y.float(), torch.nn.functional.gelu(z, approximate="tanh"), **tol)
    y, _ = g.linear(x, w, b, g.EPI_RELU, False)
    torch.testing.assert_close(y.float(), torch.relu(z), **tol)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (264, 520, 128), (1000, 1032, 2048)])
@pytest.mark.parametrize("a_kmajor,b_kmajor", [(True, True), (True, False), (False, True), (False, False)])
def test_gpu_gemm256_layouts(m, n, k, a_kmajor, b_kmajor, monkeypatch):
    """256-tile kernel forced on every operand-major combination (dgrad / wgrad use m-major
    operands read with swizzled ds_read_b64_tr_b16)."""
    import apex

    monkeypatch.setenv("APEX_AMD_GEMM256", "force")
    g = apex._native.require("gemm").gemm
    torch.manual_seed(m + n + k)
    a = torch.randn(m * k, device="cuda").to(torch.bfloat16)
    b = torch.randn(k * n, device="cuda").to(torch.bfloat16)
    c, _ = g.matmul(a, a_kmajor, b, b_kmajor, m, n, k)
    ref = _ref_mm(a, a_kmajor, b, b_kmajor, m, n, k)
    scale = k ** 0.5
    torch.testing.assert_close(c.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(512, 256, 8192), (1000, 1032, 4096), (4096, 1024, 16384)])
@pytest.mark.parametrize("a_kmajor,b_kmajor", [(False, False), (True, True)])
@pytest.mark.parametrize("splitk", ["on", "off"])
def test_gpu_gemm_splitk(m, n, k, a_kmajor, b_kmajor, splitk, monkeypatch):
    """Few output tiles x long K (weight gradients): split-K launch (fp32 partial tiles + reduce)
    vs the unsplit kernels, both against fp32 math."""
    import apex

    if splitk == "off":
        monkeypatch.setenv("APEX_AMD_SPLITK", "off")
    g = apex._native.require("gemm").gemm
    torch.manual_seed(m + n + k)
    a = torch.randn(m * k, device="cuda").to(torch.bfloat16)
    b = torch.randn(k * n, device="cuda").to(torch.bfloat16)
    c, _ = g.matmul(a, a_kmajor, b, b_kmajor, m, n, k)
    ref = _ref_mm(a, a_kmajor, b, b_kmajor, m, n, k)
    scale = k ** 0.5
    torch.testing.assert_close(c.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (300, 520, 128), (512, 768, 192), (77, 4104, 320),
                                   (2048, 2304, 1024)])
@pytest.mark.parametrize("g8p", ["1", "0"])
def test_gpu_gemm8p_nt(m, n, k, g8p, monkeypatch):
    """Phase-pipelined 256x256 kernel for two k-major operands (APEX_AMD_GEMM8P=1, default) and
    the g256 kernel it replaces, forced on every shape: K = 1..16 tiles (prologue/tail counted
    waits), ragged M / N, every epilogue incl. the activation-gradient ones reading aux."""
    import apex

    monkeypatch.setenv("APEX_AMD_GEMM256", "force")
    monkeypatch.setenv("APEX_AMD_GEMM8P", g8p)
    g = apex._native.require("gemm").gemm
    torch.manual_seed(m + n + k)
    x = (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda") * 0.2).to(torch.bfloat16)
    b = torch.randn(n, device="cuda").to(torch.bfloat16)
    z = x.float() @ w.float().t() + b.float()
    tol = dict(atol=3e-2, rtol=3e-2)
    y, _ = g.linear(x, w, b, g.EPI_NONE, False)
    torch.testing.assert_close(y.float(), z, **tol)
    y, aux = g.linear(x, w, b, g.EPI_GELU, True)
    torch.testing.assert_close(aux.float(), z, **tol)
    torch.testing.assert_close(y.float(), torch.nn.functional.gelu(z, approximate="tanh"), **tol)
    y, _ = g.linear(x, w, b, g.EPI_RELU, False)
    torch.testing.assert_close(y.float(), torch.relu(z), **tol)
    c, _ = g.matmul(x.reshape(-1), True, w.reshape(-1), True, m, n, k)
    mm = x.float() @ w.float().t()
    torch.testing.assert_close(c.float(), mm, **tol)
    pre = torch.randn(m, n, device="cuda").to(torch.bfloat16)
    c, _ = g.matmul(x.reshape(-1), True, w.reshape(-1), True, m, n, k, g.EPI_DRELU, None, pre, False)
    torch.testing.assert_close(c.float(), mm * (pre.float() > 0), **tol)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(4096, 4096, 2048), (2304, 3072, 4096)])
def test_gpu_gemm8p_race_screen(m, n, k, monkeypatch):
    """The phase pipeline reads LDS-DMA data by counted vmcnt + barrier placement only: repeat
    the launch and require bit-identical results (a mis-placed read shows as a varying tile)
    that also match fp32 math."""
    import apex

    monkeypatch.setenv("APEX_AMD_GEMM8P", "1")
    g = apex._native.require("gemm").gemm
    torch.manual_seed(7)
    a = (torch.rand(m * k, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(n * k, device="cuda") * 2 - 1).to(torch.bfloat16)
    first, _ = g.matmul(a, True, b, True, m, n, k)
    ref = a.float().view(m, k) @ b.float().view(n, k).t()
    scale = k ** 0.5
    torch.testing.assert_close(first.float() / scale, ref / scale, atol=2e-2, rtol=2e-2)
    for _ in range(30):
        c, _ = g.matmul(a, True, b, True, m, n, k)
        assert torch.equal(c, first)


# ------------------------------------------------------------------ hipBLASLt epilogue GEMMs
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m,k,n", [(16384, 1024, 4096), (1000, 512, 2048), (3 * 512, 1024, 3072)])
def test_gpu_lt_epilogues_vs_fp32(m, k, n, dtype):
    """Each hipBLASLt epilogue GEMM (csrc/bindings/lt_epilogue.cpp) against fp32 torch math, and
    the library really has a fused kernel for the GPT-2 / BERT MLP shapes (a non-empty result:
    no silent fall back to the unfused ops)."""
    from apex import _native

    lt = _native.submodule("lt_gemm")
    assert lt is not None, "lt_gemm not built"
    torch.manual_seed(0)
    x = (torch.randn(m, k, device="cuda") * 0.5).to(dtype)
    w = (torch.randn(n, k, device="cuda") / k ** 0.5).to(dtype)
    b = (torch.randn(n, device="cuda") * 0.1).to(dtype)
    pre = x.float() @ w.float().t() + b.float()

    def close(got, ref, tol=2e-2):
        s = max(1.0, float(ref.abs().max()))
        torch.testing.assert_close(got.float() / s, ref / s, atol=tol, rtol=tol)

    r = lt.linear(x, w, b, lt.EPI_BIAS)
    assert len(r) == 1
    close(r[0], pre)
    r = lt.linear(x, w, None, lt.EPI_NONE)
    close(r[0], x.float() @ w.float().t())
    # hipBLASLt (ROCm 7.2, gfx950) ships GELU_AUX_BIAS / DGELU_BGRAD kernels for fp16 but not for
    # bf16 at these shapes (profiles/lt_probe_r03.jsonl), and its bf16 DGELU kernels compute wrong
    # dz (only the first token row matches fp32), so lt_epilogue.cpp reports them unsupported: an
    # empty result sends fused_dense to its fallback; BGRADB exists for both
    r = lt.linear(x, w, b, lt.EPI_GELU_AUX_BIAS)
    if dtype == torch.float16:
        assert len(r) == 2, "no hipBLASLt GELU_AUX_BIAS kernel for this fp16 shape"
    if r:
        close(r[1], pre)
        close(r[0], torch.nn.functional.gelu(pre, approximate="tanh"))
        aux = r[1]
    else:
        aux = pre.to(dtype)
    n2 = 1024
    w2 = (torch.randn(n2, n, device="cuda") / n ** 0.5).to(dtype)
    g = (torch.randn(m, n2, device="cuda") * 0.1).to(dtype)
    z = aux.float().requires_grad_(True)
    gz = torch.autograd.grad(torch.nn.functional.gelu(z, approximate="tanh"), z, g.float() @ w2.float())[0]
    rr = lt.dgelu_bgrad(g, w2, aux)
    if rr:
        close(rr[0], gz)
        close(rr[1], gz.sum(0), tol=3e-2)
    rd = lt.dgelu_bgrad(g, w2, aux, False)
    if dtype == torch.float16:
        assert len(rd) == 1, "no hipBLASLt DGELU kernel for this fp16 shape"
    else:
        assert not rr and not rd, "bf16 dGeLU epilogues are disabled (wrong results in this hipBLASLt)"
    if rd:
        close(rd[0], gz)
    rw = lt.wgrad_bgrad(g, x, True)
    assert len(rw) == 2, "no hipBLASLt BGRADB kernel for this shape"
    close(rw[0], g.float().t() @ x.float())
    close(rw[1], g.float().sum(0), tol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m,n", [(16384, 4096), (1000, 1024), (37, 8)])
def test_gpu_dgelu_column_sum_vs_fp32(m, n, dtype):
    """One-pass dGeLU + bias gradient (csrc/gemm/gemm_mfma.hip dgelu_colsum_partial) against fp32
    torch autograd of the tanh GeLU; the bias gradient sums the rounded dz like dz.sum(0)."""
    from apex import _native

    g = _native.require("gemm").gemm
    torch.manual_seed(0)
    dy = torch.randn(m, n, device="cuda").to(dtype)
    z = (torch.randn(m, n, device="cuda") * 2).to(dtype)
    dz, db = g.dgelu_column_sum(dy, z)
    zr = z.float().requires_grad_(True)
    gz = torch.autograd.grad(torch.nn.functional.gelu(zr, approximate="tanh"), zr, dy.float())[0]
    torch.testing.assert_close(dz.float(), gz, atol=2e-2, rtol=2e-2)
    ref_db = dz.float().sum(0)
    torch.testing.assert_close(db.float(), ref_db, atol=1e-2 * max(1.0, m ** 0.5), rtol=1e-2)
    _, db32 = g.dgelu_column_sum(dy, z, torch.float32)
    torch.testing.assert_close(db32, ref_db, atol=1e-3 * max(1.0, m ** 0.5), rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m,k,n", [(16384, 1024, 4096), (1000, 256, 1024), (300, 64, 520)])
def test_gpu_dgrad_dgelu_bgrad_epilogue(m, k, n, dtype):
    """Native dgrad GEMM with dGeLU and the bias-gradient column sums in its epilogue
    (linear_dgrad_bgrad, the reference's DGELU_BGRAD): dz vs float64 torch, db BITWISE-close to
    the fp32 sum of the stored dz, the fused sums equal to the separate dGeLU epilogue's output,
    and small shapes (no 256-tile kernel) on the column-sum pass fallback."""
    from apex import _native

    g = _native.require("gemm").gemm
    torch.manual_seed(m + n)
    dy = torch.randn(m, k, device="cuda").to(dtype)
    w = (torch.randn(k, n, device="cuda") * 0.05).to(dtype)
    z = (torch.randn(m, n, device="cuda") * 2).to(dtype)
    dz, db = g.linear_dgrad_bgrad(dy, w, g.EPI_DGELU, z, torch.float32)
    assert dz.dtype == dtype and db.dtype == torch.float32 and db.shape == (n,)
    zr = z.double().requires_grad_(True)
    ref = torch.autograd.grad(torch.nn.functional.gelu(zr, approximate="tanh"), zr, dy.double() @ w.double())[0]
    torch.testing.assert_close(dz.double(), ref, atol=3e-2, rtol=2e-2)
    assert torch.equal(dz, g.linear_dgrad(dy, w, g.EPI_DGELU, z)), "the column sums must not change dz"
    torch.testing.assert_close(db.double(), dz.double().sum(0), atol=1e-4 * max(1.0, m ** 0.5), rtol=1e-5)
    _, db16 = g.linear_dgrad_bgrad(dy, w, g.EPI_DGELU, z)
    assert db16.dtype == dtype
    torch.testing.assert_close(db16.float(), db.float(), atol=1e-2 * max(1.0, m ** 0.5), rtol=1e-2)


@pytest.mark.gpu
def test_gpu_native_column_sum_helper():
    from apex import _native

    x = torch.randn(4, 1024, 1024, device="cuda", dtype=torch.bfloat16)
    got = _native.column_sum(x, torch.bfloat16)
    torch.testing.assert_close(got.float(), x.float().sum((0, 1)), atol=0.5, rtol=1e-2)
    assert got.dtype == torch.bfloat16


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_gelu_pass(dtype):
    """The native tanh-GeLU pass of the bf16 library route against torch's tanh GeLU in fp32."""
    import apex

    g = apex._native.require("gemm").gemm
    torch.manual_seed(4)
    # ragged grid-stride tail, a multi-trip size (4 vectors per lane per trip), a single vector
    for shape in ((4099, 1024), (8192, 4096), (1, 8)):
        z = (torch.randn(*shape, device="cuda") * 3).to(dtype)
        y = g.gelu(z)
        ref = torch.nn.functional.gelu(z.float(), approximate="tanh")
        torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("trans_a,trans_b", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_lt_mm_layouts(trans_a, trans_b, dtype):
    """lt_gemm.mm (hipBLASLt, per-shape top-8 timing) against an fp32 torch product for every
    operand layout, and the dense-layer wgrad helper built on it against g^T x."""
    import apex  # noqa: F401
    from apex import _native
    from apex.fused_dense.fused_dense import wgrad_gemm

    lt = _native.require("lt_gemm").lt_gemm
    torch.manual_seed(0)
    m, n, k = 192, 320, 256
    a = torch.randn((k, m) if trans_a else (m, k), device="cuda").to(dtype)
    b = torch.randn((n, k) if trans_b else (k, n), device="cuda").to(dtype)
    r = lt.mm(a, b, trans_a, trans_b)
    assert r, "hipBLASLt has no kernel for this layout"
    ref = (a.float().t() if trans_a else a.float()) @ (b.float().t() if trans_b else b.float())
    assert r[0].shape == (m, n)
    assert float((r[0].float() - ref).norm() / ref.norm()) < 1e-2
    g = torch.randn(4096, 3072, device="cuda").to(dtype)
    x = torch.randn(4096, 1024, device="cuda").to(dtype)
    want = g.float().t() @ x.float()
    assert float((wgrad_gemm(g, x).float() - want).norm() / want.norm()) < 1e-2
