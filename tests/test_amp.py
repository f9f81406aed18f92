"""amp front-end tests (reference tests/L0/run_amp/: test_basic_casts, test_checkpointing,
test_promotion, test_cache).  CPU tier: sync-mode scaler; GPU tier: the sync-free fused path."""
import copy

import pytest
import torch
import torch.nn.functional as F
from torch import nn

import apex
from apex import amp
from apex.amp._amp_state import _amp_state
from apex.optimizers import FusedAdam, FusedSGD


def _mlp(dev="cpu", seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(32, 64), nn.ReLU(), nn.Linear(64, 10)).to(dev)


def _reset():
    _amp_state.loss_scalers = []
    h = getattr(_amp_state, "handle", None)
    if h is not None:
        h._deactivate()
        _amp_state.handle = None


@pytest.fixture(autouse=True)
def _clean():
    _reset()
    yield
    _reset()


# ------------------------------------------------------------------ O1 / O4 casting (CPU)
@pytest.mark.parametrize("low", [torch.bfloat16, torch.float16])
def test_o1_cast_lists(low):
    handle = amp.init(enabled=True, patch_type=low)
    try:
        lin = nn.Linear(16, 16)
        x = torch.randn(4, 16, requires_grad=True)
        y = lin(x)
        assert y.dtype == low
        y.float().sum().backward()
        assert x.grad.dtype == torch.float32
        z = F.softmax(torch.randn(4, 8, dtype=low), dim=1)
        assert z.dtype == torch.float32
        r = F.relu(torch.randn(4, 8, dtype=low))
        assert r.dtype == low
        a = torch.randn(4, dtype=low) + torch.randn(4)
        assert a.dtype == torch.float32  # promote
        c = torch.cat([torch.randn(2, dtype=low), torch.randn(2)])
        assert c.dtype == torch.float32  # sequence promote
        with pytest.raises(NotImplementedError):  # banned on low-precision input ...
            F.binary_cross_entropy(torch.rand(4, dtype=low), torch.rand(4, dtype=low))
        assert F.binary_cross_entropy(torch.rand(4), torch.rand(4)).dtype == torch.float32  # ... fp32 runs
        with amp.disable_casts():
            assert lin(torch.randn(2, 16)).dtype == torch.float32
    finally:
        handle._deactivate()
    assert nn.Linear(4, 4)(torch.randn(2, 4)).dtype == torch.float32


def test_o1_weight_cast_cache():
    handle = amp.init(enabled=True, patch_type=torch.bfloat16)
    try:
        lin = nn.Linear(8, 8)
        lin(torch.randn(2, 8))
        n = len(handle.cache)
        lin(torch.randn(2, 8))
        assert len(handle.cache) == n  # weight cast reused
        with torch.no_grad():
            lin.weight.add_(1.0)  # in-place update invalidates
        out = lin(torch.ones(1, 8))
        ref = F.linear(torch.ones(1, 8), lin.weight.detach(), lin.bias.detach())
        torch.testing.assert_close(out.float(), ref.float(), atol=0.1, rtol=0.05)
    finally:
        handle._deactivate()


def test_user_registry_and_decorators():
    @amp.half_function
    def f(x):
        return x

    @amp.float_function
    def g(x):
        return x

    handle = amp.init(enabled=True, patch_type=torch.float16)
    try:
        assert f(torch.randn(2)).dtype == torch.float16
        assert g(torch.randn(2, dtype=torch.float16)).dtype == torch.float32
    finally:
        handle._deactivate()


# ------------------------------------------------------------------ O2 / O5 on CPU (sync mode)
@pytest.mark.parametrize("opt_level,dtype", [("O2", torch.bfloat16), ("O5", None), ("O3", torch.bfloat16)])
def test_o2_master_weights_cpu(opt_level, dtype):
    model = _mlp()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    kw = dict(cast_model_type=dtype) if dtype is not None else {}
    if opt_level == "O3":
        kw["loss_scale"] = 1.0
    model, opt = amp.initialize(model, opt, opt_level=opt_level, verbosity=0, **kw)
    assert model[0].weight.dtype == torch.bfloat16
    x = torch.randn(8, 32)
    y = torch.randint(0, 10, (8,))
    losses = []
    for _ in range(20):
        out = model(x)
        assert out.dtype == torch.float32
        loss = F.cross_entropy(out, y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    if opt_level != "O3":
        assert all(p.dtype == torch.float32 for p in amp.master_params(opt))
        sd = model.state_dict()
        assert all(v.dtype == torch.float32 for v in sd.values())


def test_overflow_skips_and_halves_cpu():
    model = _mlp()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    x = torch.randn(8, 32)
    snap = [p.detach().clone() for p in amp.master_params(opt)]
    loss = model(x).sum() * float("inf")
    opt.zero_grad()
    with amp.scale_loss(loss, opt) as s:
        s.backward()
    opt.step()
    for a, b in zip(snap, amp.master_params(opt)):
        assert torch.equal(a, b)
    sd = amp.state_dict()
    assert list(sd.keys()) == ["loss_scaler0"]
    assert sd["loss_scaler0"]["loss_scale"] == 2.0 ** 15
    assert sd["loss_scaler0"]["unskipped"] == 0


def test_state_dict_roundtrip():
    model = _mlp()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, num_losses=2,
                                verbosity=0)
    sd = amp.state_dict()
    assert set(sd.keys()) == {"loss_scaler0", "loss_scaler1"}
    sd["loss_scaler1"]["loss_scale"] = 128.0
    sd["loss_scaler1"]["unskipped"] = 7
    amp.load_state_dict(sd)
    assert amp.state_dict()["loss_scaler1"] == {"loss_scale": 128.0, "unskipped": 7}
    with pytest.raises(RuntimeError):
        amp.load_state_dict({"bogus": {}})


def test_properties_validation():
    from apex.amp.frontend import Properties, opt_levels

    p = opt_levels["O1"](Properties())
    with pytest.raises(RuntimeError):
        p.cast_model_type = torch.float16
    with pytest.raises(RuntimeError):
        amp.initialize(_mlp(), torch.optim.SGD(_mlp().parameters(), lr=1), opt_level="O9")


def test_fp16_optimizer_cpu_resnet18_plumbing():
    """BASELINE config #1 (plumbing): ResNet-18 + legacy FP16_Optimizer on CPU, loss decreases."""
    from apex.fp16_utils import FP16_Optimizer
    from apex.models import resnet18

    torch.manual_seed(0)
    model = resnet18(num_classes=10)
    opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9), static_loss_scale=128.0,
                         verbose=False)
    x = torch.randn(4, 3, 64, 64)
    y = torch.randint(0, 10, (4,))
    losses = []
    for _ in range(6):
        loss = F.cross_entropy(model(x), y)
        opt.zero_grad()
        opt.backward(loss)
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    sd = opt.state_dict()
    assert sd["loss_scaler"]["loss_scale"] == 128.0


# ------------------------------------------------------------------ GPU: sync-free fused path
def _train(model, opt, steps, x, y, inf_at=None):
    losses = []
    for i in range(steps):
        loss = F.cross_entropy(model(x), y)
        if inf_at is not None and i == inf_at:
            loss = loss * float("inf")
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.detach())
    return [float(v) for v in losses]


@pytest.mark.gpu
@pytest.mark.parametrize("opt_cls,kw", [(FusedAdam, dict(lr=1e-3)), (FusedSGD, dict(lr=0.05, momentum=0.9))])
def test_fused_amp_matches_materialized_gpu(opt_cls, kw):
    x = torch.randn(16, 32, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    res = []
    for materialize in (True, False):
        _reset()
        model = _mlp("cuda")
        opt = opt_cls(model.parameters(), materialize_master_grads=materialize, **kw)
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
        assert _amp_state.sync_free
        _train(model, opt, 5, x, y)
        res.append([p.detach().clone() for p in amp.master_params(opt)])
        for m, mp in zip([p for p in model.parameters() if p.dtype == torch.bfloat16],
                         opt._amp_stash.all_fp32_from_fp16_params):
            torch.testing.assert_close(m.float(), mp.to(torch.bfloat16).float())
    for a, b in zip(*res):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)


@pytest.mark.gpu
def test_sync_free_overflow_skip_gpu():
    x = torch.randn(16, 32, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    model = _mlp("cuda")
    opt = FusedAdam(model.parameters(), lr=1e-3, materialize_master_grads=False)
    model, opt = amp.initialize(model, opt, opt_level="O2", verbosity=0)  # fp16, dynamic scale
    _train(model, opt, 2, x, y)
    snap = [p.detach().clone() for p in amp.master_params(opt)]
    msnap = [p.detach().clone() for p in model.parameters()]
    _train(model, opt, 1, x, y, inf_at=0)
    for a, b in zip(snap, amp.master_params(opt)):
        assert torch.equal(a, b)
    for a, b in zip(msnap, model.parameters()):
        assert torch.equal(a, b)
    sd = amp.state_dict()
    assert sd["loss_scaler0"]["loss_scale"] == 2.0 ** 15
    assert sd["loss_scaler0"]["unskipped"] == 0
    _train(model, opt, 1, x, y)
    assert amp.state_dict()["loss_scaler0"]["unskipped"] == 1
    # the device step counter did not count the skipped step
    opt.state_dict()
    assert opt.param_groups[0]["step"] == 3


@pytest.mark.gpu
def test_o2_bf16_convbn_mixed_dtype_grads_not_skipped_gpu():
    """Model with bf16 convs and fp32 (keep_batchnorm_fp32) BN params: the sync-free overflow
    probe must handle the mixed-dtype grad set (regression: a mixed list was read as one dtype
    and flagged every step as overflow)."""
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.BatchNorm2d(16), torch.nn.ReLU(),
                                torch.nn.Flatten(), torch.nn.Linear(16 * 6 * 6, 10)).cuda()
    model = model.to(memory_format=torch.channels_last)
    opt = FusedAdam(model.parameters(), lr=1e-3, materialize_master_grads=False)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    x = torch.randn(8, 3, 8, 8, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    before = [p.detach().clone() for p in model.parameters()]
    _train(model, opt, 3, x, y)
    assert amp.state_dict()["loss_scaler0"]["unskipped"] == 3
    assert all(not torch.equal(a, b) for a, b in zip(before, model.parameters()))
