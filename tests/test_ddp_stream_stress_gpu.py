"""Stream-order stress test of apex.parallel.DistributedDataParallel on the GPU (SURVEY.md 5.2:
"stream-order stress tests for DDP and the side-stream prefetch").

Two ranks share one MI355X over gloo (CUDA tensors; RCCL needs one GPU per rank, the collective
ordering logic under test is the same).  The model's gradients are analytic, so any bucket that is
reduced before its gradient landed, any stale persistent bucket, or an input consumed before the
side stream that produced it finished, changes an exact expected value.  Timing is perturbed with
device-side spin kernels (``torch.cuda._sleep``) of random length on the compute stream, on the
input-prefetch side stream and between backward and the check, and the persistent-bucket path is
the steady state (``zero_grad_buckets``, never ``grad = None``).  Reference counterpart:
tests/distributed/DDP/ddp_race_condition_test.py (CPU-side ordering only).
"""
import pytest
import torch

from tests._dist_utils import run_multiprocess


def _stress_worker(rank, world, streams, trigger, message_size):
    import random

    from apex.parallel import DistributedDataParallel as DDP

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    rng = random.Random(1234 + rank)

    class Model(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.ones(1 << 16, device=dev))
            self.b = torch.nn.Parameter(torch.ones(1 << 16, device=dev))
            self.c = torch.nn.Parameter(torch.ones(1 << 15, device=dev))
            self.d = torch.nn.Parameter(torch.ones(333, device=dev))

        def forward(self, x):
            # spin inside forward so the autograd graph's producers finish at varying times
            torch.cuda._sleep(rng.randint(0, 20000))
            n = self.c.numel()
            return ((self.a * x).sum() + (self.b * x).sum() * 2.0 + (self.c * x[:n]).sum() * 3.0
                    + (self.d * x[:333]).sum() * 5.0)

    model = Model()
    if trigger:
        kw = dict(allreduce_trigger_params=[model.a, model.c], num_allreduce_streams=streams)
    else:
        kw = dict(message_size=message_size, num_allreduce_streams=streams)
    ddp = DDP(model, **kw)
    side = torch.cuda.Stream()
    for it in range(10):
        ddp.zero_grad_buckets()
        # input produced on a side stream (the data-prefetch pattern), consumed on the main one
        with torch.cuda.stream(side):
            torch.cuda._sleep(rng.randint(0, 40000))
            x = torch.full((1 << 16,), float((rank + 1) * (it + 1)), device=dev)
        torch.cuda.current_stream().wait_stream(side)
        x.record_stream(torch.cuda.current_stream())
        loss = ddp(x)
        torch.cuda._sleep(rng.randint(0, 20000))
        loss.backward()
        torch.cuda._sleep(rng.randint(0, 20000))
        mean_x = sum((r + 1) * (it + 1) for r in range(world)) / world
        for p, scale in ((model.a, 1.0), (model.b, 2.0), (model.c, 3.0), (model.d, 5.0)):
            exp = torch.full_like(p, scale * mean_x)
            assert torch.equal(p.grad, exp), (it, p.numel(), p.grad[:4].tolist(), scale * mean_x)
            # the steady state accumulates into the persistent bucket views (zero-copy)
            owner = [b for b in ddp._buckets if any(q is p for q in b.params)][0]
            base = owner.buffer.data_ptr()
            assert base <= p.grad.data_ptr() < base + owner.buffer.numel() * owner.buffer.element_size()
    if rank == 0 and not trigger:
        assert ddp.grad_copies <= len(list(model.parameters())), ddp.grad_copies


@pytest.mark.gpu
@pytest.mark.parametrize("streams,trigger,message_size", [(3, False, 1), (1, False, 10_000_000), (2, True, 0),
                                                          (1, False, 40_000)])
def test_ddp_stream_order_stress_gpu(streams, trigger, message_size):
    run_multiprocess(_stress_worker, 2, (streams, trigger, message_size), timeout=180)
