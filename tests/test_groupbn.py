"""BatchNorm2d_NHWC (fused BN / BN+ReLU / BN+add+ReLU) numerics.

Model: reference apex/contrib/test/groupbn/test_groupbn.py (NHWC BN vs a torch reference, with
and without the fused residual add + ReLU).  GPU tests compare the gfx950 pipeline against
torch.nn.BatchNorm2d (+ add + ReLU) in fp32 math, including running statistics and the
parameter gradients, and a fused-BN ResNet against the plain one."""
import pytest
import torch

from apex.contrib.groupbn import BatchNorm2d_NHWC


def _torch_ref(x, z, bn, relu):
    y = bn(x)
    if z is not None:
        y = y + z
    return torch.relu(y) if relu else y


def test_cpu_nhwc_bn_add_relu_matches_torch():
    torch.manual_seed(0)
    x = torch.randn(4, 16, 6, 6).to(memory_format=torch.channels_last).requires_grad_(True)
    z = torch.randn(4, 16, 6, 6).to(memory_format=torch.channels_last).requires_grad_(True)
    m = BatchNorm2d_NHWC(16, fuse_relu=True, torch_channels_last=True)
    ref = torch.nn.BatchNorm2d(16)
    y = m(x, z)
    xr = x.detach().clone().requires_grad_(True)
    zr = z.detach().clone().requires_grad_(True)
    yr = _torch_ref(xr, zr, ref, True)
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(z.grad, zr.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, atol=1e-4, rtol=1e-4)


def test_cpu_fused_resnet_matches_plain():
    from apex.models import resnet18

    torch.manual_seed(0)
    a = resnet18(num_classes=10)
    b = resnet18(num_classes=10, fused_bn=True)
    b.load_state_dict(a.state_dict())
    x = torch.randn(4, 3, 64, 64).to(memory_format=torch.channels_last)
    a, b = a.to(memory_format=torch.channels_last), b.to(memory_format=torch.channels_last)
    torch.testing.assert_close(a(x), b(x), atol=2e-3, rtol=2e-3)


SHAPES = [(8, 64, 56, 56), (16, 256, 14, 14), (4, 2048, 7, 7), (2, 24, 9, 9), (64, 128, 28, 28)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", ["bn", "bn_relu", "bn_add_relu"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_gpu_bn_nhwc(shape, mode, dtype):
    import apex

    assert apex._native.available()
    torch.manual_seed(sum(shape))
    c = shape[1]
    relu = mode != "bn"
    x = (torch.randn(*shape, device="cuda") * 2 + 0.5).to(dtype).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    z = None
    if mode == "bn_add_relu":
        z = torch.randn(*shape, device="cuda").to(dtype).to(memory_format=torch.channels_last).requires_grad_(True)
    m = BatchNorm2d_NHWC(c, fuse_relu=relu, torch_channels_last=True).cuda()
    ref = torch.nn.BatchNorm2d(c).cuda()
    with torch.no_grad():
        w = torch.rand(c) + 0.5
        b = torch.randn(c) * 0.2
        m.weight.copy_(w)
        m.bias.copy_(b)
        ref.weight.copy_(w)
        ref.bias.copy_(b)
    y = m(x, z)
    assert y.dtype == dtype and y.shape == x.shape
    assert y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_(True)
    zr = z.detach().float().requires_grad_(True) if z is not None else None
    yr = _torch_ref(xr, zr, ref, relu)
    tol = 2e-4 if dtype == torch.float32 else 4e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(m.running_mean, ref.running_mean, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(m.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 10, rtol=tol * 5)
    if z is not None:
        # dz = g * [relu input > 0]: an element whose pre-activation rounds to ~0 may take the other
        # side of the mask (statistics accumulated in a different order than torch's); allow a
        # handful of such boundary flips, nothing more
        bad = (z.grad.float() - zr.grad).abs() > tol + tol * zr.grad.abs()
        assert int(bad.sum()) <= max(2, zr.numel() // 500000), int(bad.sum())
    gs = max(1.0, float(ref.weight.grad.abs().max()))
    torch.testing.assert_close(m.weight.grad / gs, ref.weight.grad / gs, atol=tol * 5, rtol=tol * 5)
    gs = max(1.0, float(ref.bias.grad.abs().max()))
    torch.testing.assert_close(m.bias.grad / gs, ref.bias.grad / gs, atol=tol * 5, rtol=tol * 5)


@pytest.mark.gpu
def test_gpu_bn_nhwc_fork_sums_two_gradients():
    """fork=True: two aliases of the output; their gradients are summed inside the backward
    reduction kernel (the residual-block path of the fused ResNet) — compared with torch BN on
    the summed gradient, and a single used alias with the plain (non-fork) backward."""
    torch.manual_seed(7)
    shape = (16, 256, 14, 14)
    x = torch.randn(*shape, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    z = torch.randn(*shape, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    z.requires_grad_(True)
    m = BatchNorm2d_NHWC(256, fuse_relu=True, torch_channels_last=True).cuda()
    ref = torch.nn.BatchNorm2d(256).cuda()
    ya, yb = m(x, z, fork=True)
    assert ya.data_ptr() == yb.data_ptr() and ya.is_contiguous(memory_format=torch.channels_last)
    g1 = torch.randn(*shape, device="cuda").to(torch.bfloat16)
    g2 = torch.randn(*shape, device="cuda").to(torch.bfloat16)
    torch.autograd.backward([ya, yb], [g1, g2])
    xr = x.detach().float().requires_grad_(True)
    zr = z.detach().float().requires_grad_(True)
    yr = _torch_ref(xr, zr, ref, True)
    yr.backward(g1.float() + g2.float())
    tol = 4e-2
    torch.testing.assert_close(ya.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 10, rtol=tol * 5)
    bad = (z.grad.float() - zr.grad).abs() > tol + tol * zr.grad.abs()
    assert int(bad.sum()) <= 2, int(bad.sum())
    gs = max(1.0, float(ref.weight.grad.abs().max()))
    torch.testing.assert_close(m.weight.grad / gs, ref.weight.grad / gs, atol=tol * 5, rtol=tol * 5)
    # one alias unused: identical to the non-fork backward
    grads = []
    for fork in (True, False):
        x.grad = z.grad = None
        m.zero_grad()
        out = m(x, z, fork=fork)
        (out[1] if fork else out).backward(g2)
        grads.append((x.grad.clone(), z.grad.clone(), m.weight.grad.clone()))
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_gpu_bn_nhwc_eval_and_deterministic():
    torch.manual_seed(3)
    x = torch.randn(32, 128, 14, 14, device="cuda").to(memory_format=torch.channels_last)
    m = BatchNorm2d_NHWC(128, fuse_relu=True, torch_channels_last=True).cuda()
    x.requires_grad_(True)
    outs = []
    for _ in range(2):
        x.grad = None
        m.zero_grad()
        y = m(x)
        y.backward(torch.ones_like(y))
        outs.append((y.detach().clone(), x.grad.clone(), m.weight.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    m.eval()
    ref = torch.nn.BatchNorm2d(128).cuda().eval()
    ref.load_state_dict(m.state_dict())
    torch.testing.assert_close(m(x.detach()), torch.relu(ref(x.detach())), atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
def test_gpu_fused_resnet50_step_matches_plain():
    from apex.models import resnet50

    torch.manual_seed(0)
    a = resnet50(num_classes=100).cuda().to(memory_format=torch.channels_last)
    b = resnet50(num_classes=100, fused_bn=True).cuda().to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    x = torch.randn(8, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
    ya, yb = a(x), b(x)
    torch.testing.assert_close(yb, ya, atol=2e-3, rtol=2e-3)
    ya.sum().backward()
    yb.sum().backward()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        # 50 train-mode BN layers on a small batch amplify fp32 summation-order differences;
        # compare whole-tensor relative error (layer4 normalises over 8x2x2 = 32 values per channel;
        # conv1 sits under all of them): allow 5e-2
        rel = float((q.grad - p.grad).norm() / p.grad.norm().clamp_min(1e-12))
        assert rel < 5e-2, (n, rel)


@pytest.mark.gpu
@pytest.mark.parametrize("two_grads", [False, True])
def test_gpu_bn_relu_bitmask_matches_recompute(two_grads):
    """Residual add+ReLU backward from the forward's 1-bit ReLU mask == mask recomputed from x, z."""
    from apex import _native

    ext = _native.require("bn_nhwc").bn_nhwc
    torch.manual_seed(0)
    m, c = 4 * 14 * 14, 256
    x = torch.randn(m, c, device="cuda", dtype=torch.bfloat16)
    z = torch.randn(m, c, device="cuda", dtype=torch.bfloat16)
    w = torch.rand(c, device="cuda") + 0.5
    b = torch.randn(c, device="cuda") * 0.1
    y, sm, si, coef, mask = ext.fwd_train(x, z, w, b, None, None, 0.1, 1e-5, True, True)
    assert mask.dtype == torch.uint8 and mask.numel() * 8 == m * c
    bits = torch.stack([(mask >> k) & 1 for k in range(8)], dim=1).reshape(m, c).bool()
    assert torch.equal(bits, y > 0)
    y_ref, _, _, _, none_mask = ext.fwd_train(x, z, w, b, None, None, 0.1, 1e-5, True, False)
    assert torch.equal(y, y_ref) and (none_mask is None or none_mask.numel() == 0)
    dy = torch.randn_like(x)
    dy2 = torch.randn_like(x) if two_grads else None
    ref = ext.bwd(dy, x, z, w, sm, si, coef, True, True, dy2)
    got = ext.bwd(dy, x, None, w, sm, si, coef, True, True, dy2, mask)
    for a, r in zip(got, ref):
        assert torch.equal(a, r)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("fork", [False, True])
def test_bn_add_bn_relu_matches_two_torch_bns(device, fork):
    """relu(bn_x(x) + bn_z(z)) — the downsampling block output — through contrib.groupbn.bn_add_bn_relu
    (one fused output pass on the GPU) against two torch BatchNorm2d in fp32: outputs, input
    gradients (two incoming gradients when forked), parameter gradients and running statistics."""
    from apex.contrib.groupbn import bn_add_bn_relu
    from apex.contrib.groupbn import batch_norm as bnm

    torch.manual_seed(1)
    C = 64
    dt = torch.bfloat16 if device == "cuda" else torch.float32
    x = (torch.randn(4, C, 7, 7, device=device) * 2 + 0.5).to(dt).to(memory_format=torch.channels_last)
    z = (torch.randn(4, C, 7, 7, device=device) - 0.3).to(dt).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    z.requires_grad_(True)
    bx = BatchNorm2d_NHWC(C, fuse_relu=True, torch_channels_last=True).to(device)
    bz = BatchNorm2d_NHWC(C, fuse_relu=False, torch_channels_last=True).to(device)
    rx, rz = torch.nn.BatchNorm2d(C).to(device), torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        for m, r, s in ((bx, rx, 0.7), (bz, rz, 1.3)):
            m.weight.copy_(torch.linspace(0.5, 1.5, C) * s)
            m.bias.copy_(torch.linspace(-0.2, 0.3, C) * s)
            r.weight.copy_(m.weight)
            r.bias.copy_(m.bias)
    calls = {"n": 0}
    orig = bnm._BnDualAddReluFunction.forward

    def counting(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    bnm._BnDualAddReluFunction.forward = staticmethod(counting)
    try:
        out = bn_add_bn_relu(x, z, bx, bz, fork=fork)
    finally:
        bnm._BnDualAddReluFunction.forward = staticmethod(orig)
    assert calls["n"] == (1 if device == "cuda" else 0)
    g1 = torch.randn(4, C, 7, 7, device=device)
    g2 = torch.randn(4, C, 7, 7, device=device)
    if fork:
        y, y2 = out
        ((y.float() * g1).sum() + (y2.float() * g2).sum()).backward()
    else:
        y = out
        (y.float() * g1).sum().backward()
    xr = x.detach().float().requires_grad_(True)
    zr = z.detach().float().requires_grad_(True)
    yr = torch.relu(rx(xr) + rz(zr))
    ((yr * g1).sum() + ((yr * g2).sum() if fork else 0)).backward()
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    for got, ref in ((x.grad, xr.grad), (z.grad, zr.grad)):
        s = max(1.0, float(ref.abs().max()))
        torch.testing.assert_close(got.float() / s, ref / s, atol=tol, rtol=tol)
    for m, r in ((bx, rx), (bz, rz)):
        torch.testing.assert_close(m.running_mean, r.running_mean, atol=1e-3, rtol=1e-3)
        torch.testing.assert_close(m.running_var, r.running_var, atol=1e-3, rtol=1e-3)
        s = max(1.0, float(r.weight.grad.abs().max()))
        torch.testing.assert_close(m.weight.grad / s, r.weight.grad / s, atol=tol, rtol=tol)
        torch.testing.assert_close(m.bias.grad / s, r.bias.grad / s, atol=tol, rtol=tol)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_bn_relu_maxpool_matches_torch(device):
    """maxpool(relu(bn(x))) — the ResNet stem — through contrib.groupbn.bn_relu_maxpool (one fused
    normalize+ReLU+pool pass on the GPU) against torch BatchNorm2d + ReLU + MaxPool2d in fp32."""
    from apex.contrib.groupbn import bn_relu_maxpool
    from apex.ops.pooling import MaxPool2dNHWC

    torch.manual_seed(3)
    C = 64
    dt = torch.bfloat16 if device == "cuda" else torch.float32
    x = (torch.randn(2, C, 29, 31, device=device) * 1.5 + 0.2).to(dt).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    bn = BatchNorm2d_NHWC(C, fuse_relu=True, torch_channels_last=True).to(device)
    ref = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-0.3, 0.3, C))
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    pool = MaxPool2dNHWC(kernel_size=3, stride=2, padding=1)
    y = bn_relu_maxpool(x, bn, pool)
    xr = x.detach().float().requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(torch.relu(ref(xr)), 3, 2, 1)
    tol = 3e-2 if dt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    (y.float() * g).sum().backward()
    (yr * g).sum().backward()
    s = max(1.0, float(xr.grad.abs().max()))
    # bf16 ties inside a window can pick another equal element: compare the gradient mass
    torch.testing.assert_close(x.grad.float().sum((0, 2, 3)) / s, xr.grad.sum((0, 2, 3)) / s, atol=tol, rtol=tol)
    if dt == torch.float32:
        torch.testing.assert_close(x.grad, xr.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    sw = max(1.0, float(ref.weight.grad.abs().max()))
    torch.testing.assert_close(bn.weight.grad / sw, ref.weight.grad / sw, atol=tol, rtol=tol)
