"""SyncBatchNorm / batch-norm kernel numerics (model: reference
tests/distributed/synced_batchnorm/single_gpu_unit_test.py — kernels vs a float64 reference —
and two_gpu_unit_test.py for the cross-rank part, covered on CPU/gloo in test_distributed_cpu).

GPU tests check every native primitive (Welford stats, forward, reduce, backward; NCHW and
c_last; fused residual-add + ReLU) against fp32/fp64 torch math, and the module against
``torch.nn.BatchNorm2d`` on torch channels_last activations."""
import pytest
import torch

from apex.ops import batchnorm as bnops
from apex.parallel import SyncBatchNorm


def _ref_forward(x, w, b, eps, channel_last, z=None, relu=False):
    dims = tuple(range(x.dim() - 1)) if channel_last else (0,) + tuple(range(2, x.dim()))
    shp = (1,) * (x.dim() - 1) + (-1,) if channel_last else (1, -1) + (1,) * (x.dim() - 2)
    xd = x.double()
    mean = xd.mean(dims)
    var = xd.var(dims, unbiased=False)
    y = (xd - mean.view(shp)) / torch.sqrt(var.view(shp) + eps) * w.double().view(shp) + b.double().view(shp)
    if z is not None:
        y = y + z.double()
    if relu:
        y = torch.relu(y)
    return y, mean, var


def test_cpu_module_channels_last_memory_matches_torch_bn():
    torch.manual_seed(0)
    x = torch.randn(4, 8, 5, 5).to(memory_format=torch.channels_last).requires_grad_(True)
    m = SyncBatchNorm(8)
    ref = torch.nn.BatchNorm2d(8)
    y = m(x)
    yr = ref(x)
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(y)
    (gx,) = torch.autograd.grad(y, x, g)
    (gxr,) = torch.autograd.grad(yr, x, g)
    torch.testing.assert_close(gx, gxr, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(m.running_mean, ref.running_mean)
    torch.testing.assert_close(m.running_var, ref.running_var)


def test_cpu_fused_relu_z_backward():
    torch.manual_seed(1)
    x = torch.randn(6, 5, 7, requires_grad=True)  # channel last (C = 7)
    z = torch.randn(6, 5, 7, requires_grad=True)
    m = SyncBatchNorm(7, channel_last=True, fuse_relu=True)
    y = m(x, z)
    y.sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    zr = z.detach().clone().requires_grad_(True)
    yr = torch.relu(torch.nn.functional.batch_norm(xr.reshape(-1, 7), None, None, m.weight, m.bias, True, 0.0,
                                                   m.eps).reshape(6, 5, 7) + zr)
    yr.sum().backward()
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(z.grad, zr.grad)


CASES = [((256, 64), True), ((64, 7, 7, 2048), True), ((31, 5, 24), True), ((3, 13, 7), True),
         ((8, 64, 28, 28), False), ((5, 12, 7, 7), False), ((2, 3, 9), False)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape,channel_last", CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_gpu_bn_primitives(shape, channel_last, dtype):
    import apex

    assert apex._native.available()
    torch.manual_seed(len(shape) * 7 + shape[-1])
    c = shape[-1] if channel_last else shape[1]
    x = (torch.randn(*shape, device="cuda") * 2 + 3).to(dtype)
    w = torch.rand(c, device="cuda") + 0.5
    b = torch.randn(c, device="cuda")
    eps = 1e-5
    mean, var = bnops.welford_mean_var(x, channel_last)
    yr, mr, vr = _ref_forward(x, w, b, eps, channel_last)
    torch.testing.assert_close(mean.double(), mr, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(var.double(), vr, atol=1e-3, rtol=1e-3)
    inv_std = torch.rsqrt(var + eps)
    y = bnops.batchnorm_forward(x, mean, inv_std, w, b, channel_last)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.double(), yr, atol=tol, rtol=tol)
    # backward vs autograd on the fp64 reference
    dy = torch.randn(*shape, device="cuda").to(dtype)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr2, _, _ = _ref_forward(xr, wr, br, eps, channel_last)
    yr2.backward(dy.double())
    sum_dy, sum_dy_xmu, gw, gb = bnops.reduce_bn(dy, x, mean, inv_std, w, channel_last)
    torch.testing.assert_close(gw.double(), wr.grad, atol=tol * 10, rtol=tol)
    torch.testing.assert_close(gb.double(), br.grad, atol=tol * 10, rtol=tol)
    count = torch.tensor([x.numel() // c], dtype=torch.int32, device="cuda")
    dx = bnops.batchnorm_backward(dy, x, mean, inv_std, w, sum_dy, sum_dy_xmu, count, channel_last)
    torch.testing.assert_close(dx.double(), xr.grad, atol=tol * 5, rtol=tol * 5)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gpu_fused_add_relu_c_last(dtype):
    torch.manual_seed(5)
    shape, c = (16, 14, 14, 256), 256
    x = torch.randn(*shape, device="cuda").to(dtype)
    z = torch.randn(*shape, device="cuda").to(dtype)
    w = torch.rand(c, device="cuda") + 0.5
    b = torch.randn(c, device="cuda") * 0.1
    eps = 1e-5
    mean, var = bnops.welford_mean_var(x, True)
    inv_std = torch.rsqrt(var + eps)
    y = bnops.batchnorm_forward(x, mean, inv_std, w, b, True, z, True)
    yr, _, _ = _ref_forward(x, w, b, eps, True, z, True)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.double(), yr, atol=tol, rtol=tol)
    dy = torch.randn(*shape, device="cuda").to(dtype)
    masked = bnops.relu_backward(dy, x, z, mean, inv_std, w, b, True)
    # fused-in-kernel masking must equal the materialized mask path
    s1, s2, gw, gb = bnops.reduce_bn(dy, x, mean, inv_std, w, True, z, b, True)
    t1, t2, hw, hb = bnops.reduce_bn(masked, x, mean, inv_std, w, True)
    torch.testing.assert_close(s1, t1, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(s2, t2, atol=1e-3, rtol=1e-4)
    count = torch.tensor([x.numel() // c], dtype=torch.int32, device="cuda")
    d1 = bnops.batchnorm_backward(dy, x, mean, inv_std, w, s1, s2, count, True, z, b, True)
    d2 = bnops.batchnorm_backward(masked, x, mean, inv_std, w, t1, t2, count, True)
    torch.testing.assert_close(d1.float(), d2.float(), atol=tol, rtol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gpu_module_channels_last_vs_torch(dtype):
    torch.manual_seed(6)
    x = torch.randn(32, 64, 28, 28, device="cuda").to(dtype).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    m = SyncBatchNorm(64).cuda()
    ref = torch.nn.BatchNorm2d(64).cuda()
    y = m(x)
    assert y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_(True)
    yr = ref(xr)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 5, rtol=tol * 5)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, atol=tol * 50, rtol=tol * 5)
    torch.testing.assert_close(m.running_var, ref.running_var, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_gpu_welford_parallel_merge():
    torch.manual_seed(7)
    parts = [torch.randn(n, 33, device="cuda") * (i + 1) + i for i, n in enumerate([100, 37, 260])]
    means = torch.stack([p.mean(0) for p in parts])
    vars_ = torch.stack([p.var(0, unbiased=False) for p in parts])
    counts = torch.tensor([p.shape[0] for p in parts], dtype=torch.int32, device="cuda")
    mean, var_u, inv_std = bnops.welford_parallel(means, vars_, counts, 1e-5)
    allx = torch.cat(parts).double()
    torch.testing.assert_close(mean.double(), allx.mean(0), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(var_u.double(), allx.var(0, unbiased=True), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(inv_std.double(), 1 / torch.sqrt(allx.var(0, unbiased=False) + 1e-5),
                               atol=1e-4, rtol=1e-4)
