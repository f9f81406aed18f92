"""hipIpc peer-memory exchange (parallel/peer_memory.py, csrc/comm/peer.hip): two ranks sharing
GPU 0 (the gloo group only carries the 64-byte IPC handles), so the push / flag-wait protocol runs
for real on one device; the 8-GPU form is the same kernel with the buffers on different GPUs."""
import pytest
import torch

from tests._dist_utils import run_multiprocess


def _exchange_worker(rank, world):
    import apex
    from apex.parallel import enable_peer_memory, get_peer_exchange

    torch.cuda.set_device(0)
    ex = enable_peer_memory(None)
    assert ex is not None and get_peer_exchange(None) is ex
    # the exchange slots are written by remote GPUs while a kernel polls them: never plain
    # coarse-grained memory (coherent only at kernel boundaries)
    assert ex.alloc_kind in ("uncached", "fine-grained"), ex.alloc_kind
    for it in range(6):
        n = 100 + 37 * it
        local = torch.arange(n, device="cuda", dtype=torch.float32) + 1000.0 * (rank + 1) + it
        out = ex.all_gather(local)
        for r in range(world):
            exp = torch.arange(n, device="cuda", dtype=torch.float32) + 1000.0 * (r + 1) + it
            torch.testing.assert_close(out[r], exp, rtol=0, atol=0)
        s = ex.all_reduce_sum(torch.full((5,), float(rank + 1), device="cuda"))
        torch.testing.assert_close(s, torch.full((5,), float(sum(range(1, world + 1))), device="cuda"))
    torch.cuda.synchronize()
    ex.check()


@pytest.mark.gpu
def test_gpu_peer_exchange_two_ranks_one_gpu():
    run_multiprocess(_exchange_worker, 2, (), timeout=180)


def _bn_group_worker(rank, world):
    import apex
    from apex.contrib.groupbn import BatchNorm2d_NHWC
    from apex.parallel import get_peer_exchange

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    full = torch.randn(8, 32, 6, 6, device="cuda")
    gy = torch.randn(8, 32, 6, 6, device="cuda")
    local = full[rank * 4:(rank + 1) * 4].clone().to(memory_format=torch.channels_last).requires_grad_(True)
    bn = BatchNorm2d_NHWC(32, fuse_relu=True, bn_group=2, torch_channels_last=True).cuda()
    assert get_peer_exchange(bn.process_group) is not None
    y = bn(local)
    (y * gy[rank * 4:(rank + 1) * 4]).sum().backward()
    ref = torch.nn.BatchNorm2d(32).cuda()
    fr = full.clone().requires_grad_(True)
    yr = torch.relu(ref(fr))
    (yr * gy).sum().backward()
    torch.testing.assert_close(y, yr[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(local.grad, fr.grad[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    get_peer_exchange(bn.process_group).check()


@pytest.mark.gpu
def test_gpu_bn_group_over_peer_memory():
    run_multiprocess(_bn_group_worker, 2, (), timeout=180)


def _bn_group_fused_worker(rank, world, peer):
    """bn_group = world through the fused NHWC kernels (_BnNHWCGroupFunction): residual add +
    ReLU with a forked output, peer memory or the collective fallback; against torch BN on the
    concatenated batch (bf16 activations, fp32 statistics)."""
    import apex
    from apex.contrib.groupbn import BatchNorm2d_NHWC
    from apex.contrib.groupbn.batch_norm import _BnNHWCGroupFunction
    from apex.parallel import get_peer_exchange

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    C = 64
    full = torch.randn(8, C, 7, 7, device="cuda")
    zf = torch.randn(8, C, 7, 7, device="cuda")
    g1 = torch.randn(8, C, 7, 7, device="cuda")
    g2 = torch.randn(8, C, 7, 7, device="cuda")
    sl = slice(rank * 4, (rank + 1) * 4)
    x = full[sl].clone().to(memory_format=torch.channels_last).requires_grad_(True)
    z = zf[sl].clone().to(memory_format=torch.channels_last).requires_grad_(True)
    bn = BatchNorm2d_NHWC(C, fuse_relu=True, bn_group=world, torch_channels_last=True, peer_memory=peer).cuda()
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-0.2, 0.2, C))
    assert (get_peer_exchange(bn.process_group) is not None) == peer
    calls = {"n": 0}
    orig = _BnNHWCGroupFunction.forward

    def counting(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    _BnNHWCGroupFunction.forward = staticmethod(counting)
    y, y_alias = bn(x, z, fork=True)
    _BnNHWCGroupFunction.forward = staticmethod(orig)
    assert calls["n"] == 1, "fused group path not taken"
    ((y * g1[sl]).sum() + (y_alias * g2[sl]).sum()).backward()
    ref = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    fr = full.clone().requires_grad_(True)
    zr = zf.clone().requires_grad_(True)
    yr = torch.relu(ref(fr) + zr)
    ((yr * g1).sum() + (yr * g2).sum()).backward()
    torch.testing.assert_close(y, yr[sl], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad, fr.grad[sl], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(z.grad, zr.grad[sl], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
    import torch.distributed as dist

    gw = bn.weight.grad.detach().cpu()
    dist.all_reduce(gw)  # local weight grads: the group sum is the full-batch grad
    torch.testing.assert_close(gw, ref.weight.grad.cpu(), rtol=1e-4, atol=1e-3)
    if peer:
        get_peer_exchange(bn.process_group).check()


@pytest.mark.gpu
@pytest.mark.parametrize("peer", [True, False])
def test_gpu_bn_group_fused_residual(peer):
    run_multiprocess(_bn_group_fused_worker, 2, (peer,), timeout=180)


def _timeout_worker(rank, world):
    """A member that arrives after the timeout: the waiting rank's output is poisoned with NaN
    (never stale), the error counter raises, and the late member still completes the round."""
    import time

    import torch.distributed as dist

    import apex
    from apex.parallel.peer_memory import PeerExchange, PeerExchangeTimeout

    torch.cuda.set_device(0)
    ex = PeerExchange(None, max_floats=64, timeout_s=0.25, poll_every=1)
    local = torch.full((16,), float(rank + 1), device="cuda")
    out = ex.all_gather(local)  # epoch 1: both present
    torch.testing.assert_close(out[1 - rank], torch.full((16,), float(2 - rank), device="cuda"))
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 1:
        time.sleep(1.5)
    out = ex.all_gather(local)  # epoch 2: rank 0 waits 0.25 s and gives up
    torch.cuda.synchronize()
    if rank == 0:
        assert torch.isnan(out).all(), "timed-out exchange must poison its output"
        with pytest.raises(PeerExchangeTimeout):
            ex.check()
    else:
        torch.testing.assert_close(out[0], torch.full((16,), 1.0, device="cuda"))
        ex.check()
    dist.barrier()


@pytest.mark.gpu
def test_gpu_peer_exchange_timeout_poisons_and_raises():
    run_multiprocess(_timeout_worker, 2, (), timeout=180)


def _forced_handshake_failure_worker(rank, world):
    """A handshake that fails on ONE member: every member agrees on the RCCL/gloo path (no hang,
    no half-enabled group), the fused group BN runs through the collective fallback with the same
    numerics, and the bench-facing path report says "rccl"."""
    import apex
    from apex.contrib.groupbn import BatchNorm2d_NHWC
    from apex.contrib.groupbn.batch_norm import _bn_group
    from apex.parallel import peer_memory

    torch.cuda.set_device(0)
    group = _bn_group(world)
    ex = peer_memory.enable_peer_memory(group, _fail_handshake=(rank == 1))
    assert ex is None and peer_memory.get_peer_exchange(group) is None
    assert peer_memory.exchange_path(group) == "rccl"
    torch.manual_seed(0)
    C = 32
    full = torch.randn(8, C, 5, 5, device="cuda")
    gy = torch.randn(8, C, 5, 5, device="cuda")
    sl = slice(rank * 4, (rank + 1) * 4)
    x = full[sl].clone().to(memory_format=torch.channels_last).requires_grad_(True)
    bn = BatchNorm2d_NHWC(C, fuse_relu=True, bn_group=world, torch_channels_last=True).cuda()
    assert bn.process_group is group and peer_memory.get_peer_exchange(group) is None
    y = bn(x)
    (y * gy[sl]).sum().backward()
    ref = torch.nn.BatchNorm2d(C).cuda()
    fr = full.clone().requires_grad_(True)
    yr = torch.relu(ref(fr))
    (yr * gy).sum().backward()
    torch.testing.assert_close(y, yr[sl], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad, fr.grad[sl], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_gpu_peer_handshake_failure_falls_back_to_collectives():
    run_multiprocess(_forced_handshake_failure_worker, 2, (), timeout=180)


def _poisoned_running_stats_worker(rank, world):
    """A timed-out exchange poisons the step's statistics with NaN but leaves the running
    statistics of the group BN untouched (stats_merge skips non-finite merges)."""
    import time

    import torch.distributed as dist

    import apex
    from apex.contrib.groupbn import BatchNorm2d_NHWC
    from apex.parallel import peer_memory

    torch.cuda.set_device(0)
    bn = BatchNorm2d_NHWC(16, fuse_relu=False, bn_group=world, torch_channels_last=True).cuda()
    ex = peer_memory.get_peer_exchange(bn.process_group)
    assert ex is not None
    ex.timeout_s = 0.25
    x = torch.randn(2, 16, 3, 3, device="cuda").to(memory_format=torch.channels_last)
    bn(x)
    torch.cuda.synchronize()
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    dist.barrier()
    if rank == 1:
        time.sleep(1.5)
    y = bn(x)
    torch.cuda.synchronize()
    if rank == 0:
        assert torch.isnan(y).all()
        torch.testing.assert_close(bn.running_mean, rm, rtol=0, atol=0)
        torch.testing.assert_close(bn.running_var, rv, rtol=0, atol=0)
    dist.barrier()


@pytest.mark.gpu
def test_gpu_peer_timeout_keeps_running_stats():
    run_multiprocess(_poisoned_running_stats_worker, 2, (), timeout=180)
