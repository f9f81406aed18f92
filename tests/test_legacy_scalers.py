"""Legacy scaling APIs: ``handle.wrap_optimizer`` (OptimWrapper, one scaler per loss; reference
apex/amp/opt.py) and the ``fp16_utils`` loss scalers (reference apex/fp16_utils/loss_scaler.py).
Expected behaviour is derived from the reference's documented semantics, recomputed by hand."""
import pytest
import torch

from apex.amp.handle import AmpHandle, NoOpHandle
from apex.fp16_utils import DynamicLossScaler, LossScaler


def _model():
    torch.manual_seed(0)
    return torch.nn.Linear(4, 3)


def test_optim_wrapper_two_losses_sum_unscaled_grads():
    m = _model()
    ref = _model()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    w = AmpHandle().wrap_optimizer(opt, num_loss=2)
    x = torch.randn(5, 4)
    for it in range(3):
        w.zero_grad()
        with w.scale_loss(m(x).pow(2).sum()) as s:
            assert float(s.detach()) > 1000.0  # scaled by the dynamic scale (2^16)
            s.backward()
        with w.scale_loss(m(x).sum() * 3.0) as s:
            s.backward()
        w.step()
        ref_opt.zero_grad()
        (ref(x).pow(2).sum() + ref(x).sum() * 3.0).backward()
        ref_opt.step()
        for a, b in zip(m.parameters(), ref.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_optim_wrapper_overflow_in_one_loss_skips_step_and_backs_off():
    m = _model()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    w = AmpHandle().wrap_optimizer(opt, num_loss=2)
    before = [p.detach().clone() for p in m.parameters()]
    x = torch.randn(5, 4)
    with w.scale_loss(m(x).sum()) as s:
        s.backward()
    with w.scale_loss(m(x).sum() * float("inf")) as s:
        s.backward()
    assert w.step() is None
    for a, b in zip(m.parameters(), before):
        assert torch.equal(a, b), "overflowed step must not update"
    assert w._scalers[0].loss_scale() == 2.0 ** 16  # clean loss keeps its scale
    assert w._scalers[1].loss_scale() == 2.0 ** 15  # overflowed loss backs off
    # next step is clean again and applies
    w.zero_grad()
    with w.scale_loss(m(x).sum()) as s:
        s.backward()
    with w.scale_loss(m(x).sum()) as s:
        s.backward()
    w.step()
    assert not all(torch.equal(a, b) for a, b in zip(m.parameters(), before))


def test_optim_wrapper_too_many_losses_raises():
    m = _model()
    w = AmpHandle().wrap_optimizer(torch.optim.SGD(m.parameters(), lr=0.1), num_loss=1)
    with w.scale_loss(m(torch.randn(2, 4)).sum()) as s:
        s.backward()
    with pytest.raises(RuntimeError):
        with w.scale_loss(m(torch.randn(2, 4)).sum()) as s:
            s.backward()


def test_optim_wrapper_inactive_handle_is_passthrough():
    m = _model()
    w = NoOpHandle().wrap_optimizer(torch.optim.SGD(m.parameters(), lr=0.1))
    loss = m(torch.randn(2, 4)).sum()
    with w.scale_loss(loss) as s:
        assert s is loss


def test_dynamic_loss_scaler_schedule():
    s = DynamicLossScaler(init_scale=2.0 ** 10, scale_factor=2.0, scale_window=3)
    assert s.last_overflow_iter == -1
    seq = []
    for overflow in [False, False, False, False, True, False, False, False, True, True]:
        s.update_scale(overflow)
        seq.append(s.loss_scale)
    # grows after 3 clean steps, halves on every overflow, the window restarts after one
    assert seq == [1024, 1024, 2048, 2048, 1024, 1024, 1024, 2048, 1024, 512]
    assert s.cur_iter == 10 and s.last_overflow_iter == 9
    s.last_overflow_iter = 7
    assert s.last_overflow_iter == 7


def test_dynamic_loss_scaler_floor_and_overflow_detection():
    s = DynamicLossScaler(init_scale=2.0, scale_window=100)
    for _ in range(4):
        s.update_scale(True)
    assert s.loss_scale == 1
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.tensor([1.0, 2.0, 3.0])
    q = torch.nn.Parameter(torch.ones(2))
    assert not s.has_overflow([p, q])  # q has no grad
    p.grad[1] = float("nan")
    assert s.has_overflow([p, q])
    assert DynamicLossScaler._has_inf_or_nan(torch.tensor([0.0, float("-inf")]))
    assert not DynamicLossScaler._has_inf_or_nan(torch.zeros(4, dtype=torch.float16))


def test_static_loss_scaler():
    s = LossScaler(128.0)
    assert s.loss_scale == 128.0 and not s.has_overflow([]) and s.update_scale(True) is None
    m = _model()
    x = torch.randn(3, 4)
    s.backward(m(x).sum())
    g = m.weight.grad.clone()
    m.zero_grad()
    m(x).sum().backward()
    torch.testing.assert_close(g, m.weight.grad * 128.0)
    gi = (torch.ones(2), None)
    out = s.scale_gradient(None, gi, None)
    assert torch.equal(out[0], torch.full((2,), 128.0)) and out[1] is None
