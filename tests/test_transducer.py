"""RNN-T transducer joint / loss.

Model: reference apex/contrib/test/transducer/test_transducer_joint.py (joint vs f+g broadcast,
packed and unpacked, relu / dropout masks, f/g grads) and test_transducer_loss.py (loss and
grad vs a python alpha recursion).  GPU tiers compare the gfx950 kernels with fp32 torch math."""
import pytest
import torch
import torch.nn.functional as F

from apex.contrib.transducer import TransducerJoint, TransducerLoss
from apex.contrib.transducer.transducer import _loss_ref


def _data(dev, dtype=torch.float32, B=3, T=7, U=5, H=16, V=11):
    torch.manual_seed(0)
    f_len = torch.tensor([7, 4, 6], dtype=torch.int32, device=dev)
    y_len = torch.tensor([4, 2, 3], dtype=torch.int32, device=dev)
    f = torch.randn(B, T, H, device=dev, dtype=dtype, requires_grad=True)
    g = torch.randn(B, U, H, device=dev, dtype=dtype, requires_grad=True)
    x = torch.randn(B, T, U, V, device=dev, dtype=dtype, requires_grad=True)
    label = torch.randint(1, V, (B, U - 1), dtype=torch.int32, device=dev)
    return f, g, f_len, y_len, x, label


def _joint_ref(f, g, f_len, g_len):
    h = f.float().unsqueeze(2) + g.float().unsqueeze(1)
    B, T, U = h.shape[:3]
    valid = (torch.arange(T, device=f.device).view(1, T, 1) < f_len.view(B, 1, 1)) & \
            (torch.arange(U, device=f.device).view(1, 1, U) < g_len.view(B, 1, 1))
    return h, valid


@pytest.mark.parametrize("relu", [False, True])
def test_cpu_joint(relu):
    f, g, f_len, y_len, _, _ = _data("cpu")
    g_len = y_len + 1
    joint = TransducerJoint(relu=relu)
    out = joint(f, g, f_len, g_len)
    h, valid = _joint_ref(f, g, f_len, g_len)
    ref = torch.where(valid.unsqueeze(-1), torch.relu(h) if relu else h, torch.full_like(h, -1.0))
    torch.testing.assert_close(out, ref)
    gr = torch.randn_like(out)
    out.backward(gr)
    m = valid.unsqueeze(-1) & ((h > 0) if relu else torch.ones_like(h, dtype=torch.bool))
    torch.testing.assert_close(f.grad, (gr * m).sum(2))
    torch.testing.assert_close(g.grad, (gr * m).sum(1))


def test_cpu_loss_matches_ctc_style_reference():
    _, _, f_len, y_len, x, label = _data("cpu")
    loss = TransducerLoss()(x, label, f_len, y_len, 0)
    assert loss.shape == (3,) and torch.isfinite(loss).all() and (loss > 0).all()
    loss.sum().backward()
    # gradient of the NLL wrt logits sums to zero over the vocabulary at every valid lattice point
    torch.testing.assert_close(x.grad.sum(-1), torch.zeros_like(x.grad.sum(-1)), atol=1e-5, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("relu,pack", [(False, False), (True, False), (False, True), (True, True)])
def test_gpu_joint(dtype, relu, pack):
    f, g, f_len, y_len, _, _ = _data("cuda", dtype, H=64)
    g_len = y_len + 1
    B, T, H = f.shape
    U = g.size(1)
    joint = TransducerJoint(pack_output=pack, relu=relu)
    bo = torch.cumsum(f_len * g_len, 0).long()
    out = joint(f, g, f_len, g_len, batch_offset=bo, packed_batch=int(bo[-1]))
    h, valid = _joint_ref(f, g, f_len, g_len)
    act = torch.relu(h) if relu else h
    ref = torch.where(valid.unsqueeze(-1), act, torch.full_like(h, -1.0))
    gr_full = torch.randn(B, T, U, H, device="cuda")
    if pack:
        rows = [ref[b, :int(f_len[b]), :int(g_len[b])].reshape(-1, H) for b in range(B)]
        grows = [gr_full[b, :int(f_len[b]), :int(g_len[b])].reshape(-1, H) for b in range(B)]
        ref, gr = torch.cat(rows), torch.cat(grows)
    else:
        gr = gr_full
    tol = dict(atol=1e-2, rtol=1e-2) if dtype == torch.float16 else dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out.float(), ref, **tol)
    out.backward(gr.to(dtype))
    m = valid.unsqueeze(-1) & ((h > 0) if relu else torch.ones_like(h, dtype=torch.bool))
    g_eff = gr_full * m
    torch.testing.assert_close(f.grad.float(), g_eff.sum(2), **tol)
    torch.testing.assert_close(g.grad.float(), g_eff.sum(1), **tol)


@pytest.mark.gpu
def test_gpu_joint_dropout_mask_probe():
    f, g, f_len, y_len, _, _ = _data("cuda", torch.float32, H=64)
    joint = TransducerJoint(relu=True, dropout=True, dropout_prob=0.3, probe_mask=True)
    joint.train()
    out = joint(f, g, f_len, y_len + 1)
    mask = joint.mask_probe[0].bool()
    h, valid = _joint_ref(f, g, f_len, y_len + 1)
    ref = torch.where(mask, h / 0.7, torch.zeros_like(h))
    ref = torch.where(valid.unsqueeze(-1), ref, torch.full_like(h, -1.0))
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    kept = mask[valid.unsqueeze(-1).expand_as(mask) & (h > 0)].float().mean().item()
    assert abs(kept - 0.7) < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_gpu_loss(fused, dtype):
    _, _, f_len, y_len, x, label = _data("cuda", dtype, V=37)
    loss = TransducerLoss(fuse_softmax_backward=fused)(x, label, f_len, y_len, 0)
    xr = x.detach().float().cpu().requires_grad_(True)
    ref = _loss_ref(F.log_softmax(xr, -1), label.cpu(), f_len.cpu(), y_len.cpu(), 0)
    tol = dict(atol=2e-2, rtol=2e-3) if dtype == torch.float16 else dict(atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(loss.float().cpu(), ref.detach(), **tol)
    lg = torch.rand(3, device="cuda")
    loss.backward(lg.to(loss.dtype))
    ref.backward(lg.cpu())
    B, T, U = 3, 7, 5
    valid = (torch.arange(T).view(1, T, 1) < f_len.cpu().view(B, 1, 1)) & \
            (torch.arange(U).view(1, 1, U) < (y_len.cpu() + 1).view(B, 1, 1))
    got = x.grad.float().cpu() * valid.unsqueeze(-1)
    torch.testing.assert_close(got, xr.grad * valid.unsqueeze(-1), **tol)


@pytest.mark.gpu
def test_gpu_loss_packed():
    _, _, f_len, y_len, x, label = _data("cuda", torch.float32, V=37)
    loss_full = TransducerLoss()(x, label, f_len, y_len, 0)
    B, T, U, V = x.shape
    rows = [x.detach()[b, :int(f_len[b]), :int(y_len[b]) + 1].reshape(-1, V) for b in range(B)]
    xp = torch.cat(rows).requires_grad_(True)
    bo = torch.cumsum(f_len * (y_len + 1), 0).long()
    loss_p = TransducerLoss(packed_input=True)(xp, label, f_len, y_len, 0, batch_offset=bo, max_f_len=T)
    torch.testing.assert_close(loss_p, loss_full, atol=1e-5, rtol=1e-5)
    loss_p.sum().backward()
    loss_full.sum().backward()
    gref = torch.cat([x.grad[b, :int(f_len[b]), :int(y_len[b]) + 1].reshape(-1, V) for b in range(B)])
    torch.testing.assert_close(xp.grad, gref, atol=1e-5, rtol=1e-5)
