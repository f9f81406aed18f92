"""LARC wrapper (apex.parallel.LARC; reference apex/parallel/LARC.py, tests/L0/run_amp/test_larc.py):
per-tensor trust ratio with clip / scale modes, weight decay absorbed, against the math written
out per tensor; the GPU variant runs the multi-tensor-norm path."""
import copy

import pytest
import torch


def _reference_step(params, lr, wd, trust, clip, eps, momentum_buf, momentum):
    with torch.no_grad():
        for p in params:
            if p.grad is None:
                continue
            pn, gn = p.norm(), p.grad.norm()
            if pn != 0 and gn != 0:
                r = trust * pn / (gn + pn * wd + eps)
                if clip:
                    r = min(r / lr, 1.0)
                g = (p.grad + wd * p) * r
            else:
                g = p.grad.clone()
            buf = momentum_buf.setdefault(id(p), torch.zeros_like(p))
            buf.mul_(momentum).add_(g)
            p.sub_(lr * buf)


def _run(device, clip):
    from apex.parallel import LARC

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(12, 24), torch.nn.ReLU(), torch.nn.Linear(24, 3)).to(device)
    ref = copy.deepcopy(model)
    opt = LARC(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-3), trust_coefficient=0.02,
               clip=clip)
    bufs = {}
    for it in range(4):
        x = torch.randn(16, 12, device=device)
        y = torch.randn(16, 3, device=device)
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
        for p in ref.parameters():
            p.grad = None
        torch.nn.functional.mse_loss(ref(x), y).backward()
        _reference_step(list(ref.parameters()), 0.1, 1e-3, 0.02, clip, 1e-8, bufs, 0.9)
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    # weight decay restored after every step; delegation works
    assert opt.param_groups[0]["weight_decay"] == 1e-3
    assert "state" in opt.state_dict()


@pytest.mark.parametrize("clip", [True, False])
def test_larc_matches_reference(clip):
    _run("cpu", clip)


@pytest.mark.gpu
@pytest.mark.parametrize("clip", [True, False])
def test_gpu_larc_matches_reference(clip):
    _run("cuda", clip)
