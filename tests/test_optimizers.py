"""Fused optimizers vs reference optimizers (pattern of reference
tests/L0/run_optimizers/test_fused_optimizer.py:63-85: identical params, 7 steps, compare).

CPU runs exercise the torch reference path of every amp_C op; GPU runs exercise the gfx950
kernels (including the sync-free capturable variants)."""
import math

import pytest
import torch

import apex  # noqa: F401
from apex.optimizers import FusedAdagrad, FusedAdam, FusedLAMB, FusedNovoGrad, FusedSGD

SHAPES = [(278011,), (17, 33), (1,), (65536 + 7,)]


def _params(dev, dtype=torch.float32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(dev, dtype)) for s in SHAPES]


def _grads(params, it):
    g = torch.Generator().manual_seed(100 + it)
    for p in params:
        p.grad = torch.randn(p.shape, generator=g).to(p.device, p.dtype)


def _run(ref_cls, ref_kw, fused_cls, fused_kw, dev, dtype=torch.float32, iters=7):
    ref_p = _params(dev, dtype)
    tst_p = _params(dev, dtype)
    ref_opt = ref_cls(ref_p, **ref_kw)
    tst_opt = fused_cls(tst_p, **fused_kw)
    for it in range(iters):
        _grads(ref_p, it)
        _grads(tst_p, it)
        ref_opt.step()
        tst_opt.step()
    return ref_p, tst_p


def _devs():
    devs = ["cpu"]
    if torch.cuda.is_available():
        devs.append("cuda")
    return devs


@pytest.mark.parametrize("adam_w_mode", [True, False])
@pytest.mark.parametrize("dev", _devs())
def test_fused_adam(adam_w_mode, dev):
    ref_cls = torch.optim.AdamW if adam_w_mode else torch.optim.Adam
    kw = dict(lr=5e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.05)
    ref_p, tst_p = _run(ref_cls, kw, FusedAdam, dict(kw, adam_w_mode=adam_w_mode), dev)
    for r, t in zip(ref_p, tst_p):
        torch.testing.assert_close(t, r, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("nesterov", [False, True])
@pytest.mark.parametrize("dev", _devs())
def test_fused_sgd(nesterov, dev):
    kw = dict(lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=nesterov)
    ref_p, tst_p = _run(torch.optim.SGD, kw, FusedSGD, kw, dev)
    for r, t in zip(ref_p, tst_p):
        torch.testing.assert_close(t, r, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("dev", _devs())
def test_fused_adagrad(dev):
    kw = dict(lr=0.05, eps=1e-10, weight_decay=1e-3)
    ref_p, tst_p = _run(torch.optim.Adagrad, kw, FusedAdagrad, kw, dev)
    for r, t in zip(ref_p, tst_p):
        torch.testing.assert_close(t, r, atol=1e-5, rtol=1e-4)


class RefLAMB(torch.optim.Optimizer):
    """In-test LAMB (as the reference's tests/L0/run_optimizers/test_lamb.py does)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.max_grad_norm = max_grad_norm

    @torch.no_grad()
    def step(self):
        gn = torch.sqrt(sum((p.grad.float() ** 2).sum() for g in self.param_groups for p in g["params"]))
        clip = gn / self.max_grad_norm if gn > self.max_grad_norm else 1.0
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["m"] = torch.zeros_like(p)
                    st["v"] = torch.zeros_like(p)
                st["step"] += 1
                g = p.grad / clip
                st["m"].mul_(b1).add_(g, alpha=1 - b1)
                st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
                mh = st["m"] / (1 - b1 ** st["step"])
                vh = st["v"] / (1 - b2 ** st["step"])
                upd = mh / (vh.sqrt() + group["eps"]) + group["weight_decay"] * p
                pn, un = p.norm(), upd.norm()
                ratio = pn / un if (pn > 0 and un > 0) else 1.0
                p.add_(upd * (-group["lr"] * ratio))


@pytest.mark.parametrize("dev", _devs())
def test_fused_lamb(dev):
    kw = dict(lr=1e-2, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, max_grad_norm=1.0)
    ref_p, tst_p = _run(RefLAMB, kw, FusedLAMB, kw, dev)
    for r, t in zip(ref_p, tst_p):
        torch.testing.assert_close(t, r, atol=2e-5, rtol=2e-4)


@pytest.mark.parametrize("dev", _devs())
def test_fused_novograd_runs(dev):
    ps = _params(dev)
    opt = FusedNovoGrad(ps, lr=1e-2, weight_decay=1e-3)
    before = [p.detach().clone() for p in ps]
    for it in range(3):
        _grads(ps, it)
        opt.step()
    assert all(not torch.equal(b, p) for b, p in zip(before, ps))
    assert all(torch.isfinite(p).all() for p in ps)
    assert opt.param_groups[0]["exp_avg_sq"][1].numel() == len(ps)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_adam_low_precision_params_gpu(dtype):
    kw = dict(lr=5e-4, weight_decay=0.0)
    ref_p = _params("cuda", torch.float32)
    tst_p = _params("cuda", dtype)
    ref_opt = torch.optim.AdamW(ref_p, **kw)
    tst_opt = FusedAdam(tst_p, **kw)
    for it in range(5):
        _grads(ref_p, it)
        for r, t in zip(ref_p, tst_p):
            t.grad = r.grad.to(dtype)
        ref_opt.step()
        tst_opt.step()
    for r, t in zip(ref_p, tst_p):
        torch.testing.assert_close(t.float(), r, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
def test_adam_capturable_matches_plain_gpu():
    """The sync-free kernel (device lr/step/inv_scale, depth-5 model copy) == plain kernel."""
    import amp_C

    p1 = _params("cuda")
    p2 = [p.detach().clone() for p in p1]
    m1 = [torch.zeros_like(p) for p in p1]
    v1 = [torch.zeros_like(p) for p in p1]
    m2 = [torch.zeros_like(p) for p in p1]
    v2 = [torch.zeros_like(p) for p in p1]
    model = [p.detach().to(torch.bfloat16) for p in p1]
    noop = torch.zeros(1, dtype=torch.int32, device="cuda")
    step_t = torch.zeros(1, device="cuda")
    lr_t = torch.full((1,), 1e-3, device="cuda")
    inv = torch.full((1,), 1.0 / 1024, device="cuda")
    for it in range(1, 4):
        g = [torch.randn_like(p) for p in p1]
        gs = [x * 1024 for x in g]
        amp_C.multi_tensor_adam(65536, noop, [g, [p.data for p in p1], m1, v1], 1e-3, 0.9, 0.999, 1e-8, it, 1, 1, 0.01)
        step_t += 1
        amp_C.multi_tensor_adam_capturable(65536, noop, [gs, [p.data for p in p2], m2, v2, model], lr_t, 0.9, 0.999,
                                           1e-8, step_t, 1, 1, 0.01, inv)
    for a, b, mm in zip(p1, p2, model):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)
        torch.testing.assert_close(mm.float(), b.to(torch.bfloat16).float())
    # skip flag set -> nothing changes
    snap = [p.detach().clone() for p in p2]
    noop.fill_(1)
    amp_C.multi_tensor_adam_capturable(65536, noop, [gs, [p.data for p in p2], m2, v2, model], lr_t, 0.9, 0.999, 1e-8,
                                       step_t, 1, 1, 0.01, inv)
    for a, b in zip(snap, p2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_adam_capturable_resume_continues_bias_correction(dev):
    """save -> load -> continue equals uninterrupted training (the device step counter is seeded
    from the checkpointed step, so bias correction does not restart)."""
    from apex.optimizers import FusedAdam

    def params():
        torch.manual_seed(0)
        return [torch.nn.Parameter(torch.randn(257, device=dev)), torch.nn.Parameter(torch.randn(33, 7, device=dev))]

    def grads(i, ps):
        g = torch.Generator(device="cpu").manual_seed(100 + i)
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g).to(dev)

    ref_p = params()
    ref = FusedAdam(ref_p, lr=1e-2, capturable=True)
    for i in range(5):
        grads(i, ref_p)
        ref.step()
    a_p = params()
    a = FusedAdam(a_p, lr=1e-2, capturable=True)
    for i in range(3):
        grads(i, a_p)
        a.step()
    sd = a.state_dict()
    assert sd["param_groups"][0]["step"] == 3
    b_p = [torch.nn.Parameter(p.detach().clone()) for p in a_p]
    b = FusedAdam(b_p, lr=1e-2, capturable=True)
    b.load_state_dict(sd)
    for i in range(3, 5):
        grads(i, b_p)
        b.step()
    for x, y in zip(b_p, ref_p):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
