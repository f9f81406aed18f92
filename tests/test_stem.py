"""The native ResNet stem (csrc/conv/stem.hip, ops/stem.py): 7x7/2 conv + BN statistics,
BN + ReLU + 3x3/2 max pool, the fused pool/BN backward reduction and the weight gradient with
the BN-backward prologue, each against a float64 PyTorch reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

SHAPES = [
    # n, cin, h, w
    (2, 3, 32, 32),
    (3, 3, 37, 30),   # odd rows: the last pooled row's window runs past the map
    (1, 4, 20, 26),
    (1, 1, 15, 17),
]


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _ext():
    from apex import _native

    return _native.require("conv").conv


def _pool_ref(y, coef):
    """bf16-rounded relu(bn(y)) pooled with torch's first-maximum rule; window indices kh*3+kw."""
    c = y.size(1)
    sc = coef[:c].double().view(1, c, 1, 1)
    sh = coef[c:].double().view(1, c, 1, 1)
    r = torch.relu((y.double() * sc + sh).float()).to(y.dtype).float()
    p, flat = F.max_pool2d(r, 3, 2, 1, return_indices=True)
    return r, p, flat


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,h,w", SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_stem_kernels_match_float64(n, cin, h, w, dtype):
    import apex  # noqa: F401

    torch.manual_seed(0)
    dev = "cuda"
    ext = _ext()
    x = torch.randn(n, cin, h, w, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(64, cin, 7, 7, device=dev) * 0.2).to(dtype).contiguous(memory_format=torch.channels_last)
    g = torch.rand(64, device=dev) + 0.5
    b = torch.randn(64, device=dev) * 0.2
    rm = torch.randn(64, device=dev) * 0.1
    rv = torch.rand(64, device=dev) + 0.5
    eps, mom = 1e-5, 0.1

    # conv + statistics
    y, part, xp = ext.stem_fprop(x, wt, rm)
    ref_y = F.conv2d(x.double(), wt.double(), None, 2, 3)
    assert y.shape == ref_y.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref_y) < 8e-3
    m = y.size(0) * y.size(2) * y.size(3)
    rm2, rv2 = rm.clone(), rv.clone()
    sm, si, coef = ext.bn_finalize(part, float(m), rm2, g, b, rm2, rv2, eps, mom)
    yd = y.double()
    mean = yd.mean((0, 2, 3))
    var = yd.var((0, 2, 3), unbiased=False)
    assert _rel(sm, mean) < 1e-5
    assert _rel(si, (var + eps).rsqrt()) < 1e-4
    assert _rel(rm2, (1 - mom) * rm.double() + mom * mean) < 1e-5
    assert _rel(rv2, (1 - mom) * rv.double() + mom * var * m / (m - 1)) < 1e-4

    # BN + ReLU + pool
    p, idx = ext.stem_pool(y, coef)
    r, ref_p, flat = _pool_ref(y, coef)
    assert p.shape == ref_p.shape
    assert torch.equal(p.float(), ref_p)
    ow = y.size(3)
    ph, pw = p.size(2), p.size(3)
    ih = flat // ow - (torch.arange(ph, device=dev).view(1, 1, ph, 1) * 2 - 1)
    iw = flat % ow - (torch.arange(pw, device=dev).view(1, 1, 1, pw) * 2 - 1)
    assert torch.equal(idx.permute(0, 3, 1, 2).long(), ih * 3 + iw)

    # backward: float64 autograd through the same argmax choice
    dp = torch.randn(p.shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
    yv = yd.clone().requires_grad_(True)
    gd, bd = g.double().requires_grad_(True), b.double().requires_grad_(True)
    mu = yv.mean((0, 2, 3), keepdim=True)
    va = yv.var((0, 2, 3), unbiased=False, keepdim=True)
    o = torch.relu((yv - mu) / (va + eps).sqrt() * gd.view(1, -1, 1, 1) + bd.view(1, -1, 1, 1))
    pooled = o.flatten(2).gather(2, flat.flatten(2)).view_as(ref_p)
    (pooled * dp.double()).sum().backward()

    part2 = ext.stem_reduce(dp, idx, y, coef, sm)
    cb, gg, gb = ext.bnbwd_finalize(part2, float(m), sm, si, g)
    assert _rel(gg, gd.grad) < 1e-4
    assert _rel(gb, bd.grad) < 1e-4
    dw = ext.stem_wgrad(dp, idx, y, coef, cb.view(-1), xp, wt)
    assert dw.shape == wt.shape and dw.dtype == wt.dtype and dw.stride() == wt.stride()
    ref_dw = torch.nn.grad.conv2d_weight(x.double(), wt.shape, yv.grad, 2, 3)
    assert _rel(dw, ref_dw) < 1.5e-2


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16])
def test_gpu_stem_node_matches_module_path(dtype):
    """ResNet stem through ops/stem.py vs the module path (channel-padded conv, fused NHWC BN
    + pool) with the same weights: output, parameter gradients and running statistics.  Both
    are bf16 paths that round the BN-input gradient differently before a cancelling weight-
    gradient sum (6 % apart per element at this size); the exact-arithmetic check of every
    kernel is test_gpu_stem_kernels_match_float64."""
    import copy

    import apex  # noqa: F401
    from apex.models.resnet import resnet50
    from apex.ops import stem

    torch.manual_seed(1)
    model = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    model.conv1.to(dtype)
    ref = copy.deepcopy(model)
    x = torch.randn(4, 3, 64, 64, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    assert stem.stem_supported(model.conv1, model.bn1, model.maxpool, x)
    out = stem.stem_forward(model.conv1, model.bn1, model.maxpool, x)
    from apex.contrib.groupbn import bn_relu_maxpool

    want = bn_relu_maxpool(ref.conv1(x), ref.bn1, ref.maxpool)
    assert out.shape == want.shape
    assert _rel(out, want) < 2e-2
    gout = torch.randn_like(want)
    out.backward(gout)
    want.backward(gout)
    assert _rel(model.conv1.weight.grad, ref.conv1.weight.grad) < 1e-1
    assert _rel(model.bn1.weight.grad, ref.bn1.weight.grad) < 5e-2
    assert _rel(model.bn1.bias.grad, ref.bn1.bias.grad) < 5e-2
    assert _rel(model.bn1.running_mean, ref.bn1.running_mean) < 1e-2
    assert _rel(model.bn1.running_var, ref.bn1.running_var) < 1e-2


def test_stem_unsupported_on_cpu():
    from apex.models.resnet import resnet50
    from apex.ops import stem

    model = resnet50(fused_bn=True)
    x = torch.randn(1, 3, 32, 32)
    assert not stem.stem_supported(model.conv1, model.bn1, model.maxpool, x)


@pytest.mark.gpu
def test_gpu_o2_fp32_batch_cast_in_the_stem_pad_is_bitwise_the_amp_cast():
    """amp O2 leaves the fused-BN ResNet's input cast to its stem (models/resnet.py
    _amp_casts_input): the padding pass rounds the fp32 batch to bf16 exactly as ``.to()`` does,
    so the forward (the loss) and the classifier gradients equal those of a batch cast before the
    call bitwise; deeper gradients agree to run-to-run noise."""
    import copy

    from apex import amp
    from apex.models.resnet import resnet50
    from apex.optimizers import FusedAdam

    torch.manual_seed(3)
    base = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 1000, (8,), device="cuda")
    results = []
    for pre_cast in (False, True):
        model = copy.deepcopy(base)
        opt = FusedAdam(model.parameters(), lr=1e-3)
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16,
                                    keep_batchnorm_fp32=True, verbosity=0)
        inp = x.to(torch.bfloat16) if pre_cast else x
        loss = torch.nn.functional.cross_entropy(model(inp), t)
        loss.backward()
        results.append((loss.detach(), [model.fc.weight.grad.clone(), model.fc.bias.grad.clone()],
                        [p.grad.clone() for p in model.parameters() if p.grad is not None]))
    (l0, fc0, g0), (l1, fc1, g1) = results
    assert torch.equal(l0, l1)
    # the classifier's gradients depend only on the (bitwise equal) forward
    assert all(torch.equal(a, b) for a, b in zip(fc0, fc1))
    # deeper gradients pass the library stride-2 data gradient (not bitwise reproducible run to
    # run; bf16 BN-bias sums cancel heavily): same size, finite, loosely equal
    assert len(g0) == len(g1)
    for a, b in zip(g0, g1):
        assert torch.isfinite(a).all() and _rel(a, b) < 0.25
