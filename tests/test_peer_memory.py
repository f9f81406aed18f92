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
