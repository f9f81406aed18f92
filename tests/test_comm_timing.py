"""Collective accounting (apex.parallel.comm_timing): DDP's exposed tail all-reduce and the
synchronized batch norm's statistics exchange are recorded as spans per step, so a multi-GPU
bench line reports allreduce_exposed_ms / bn_exchange_ms_per_step.  gloo, world 2, CPU."""
import torch

from tests._dist_utils import run_multiprocess


def _worker(rank, world):
    import torch.distributed as dist

    import apex
    from apex.contrib.groupbn.batch_norm import _exchange_gather, _exchange_sum
    from apex.parallel import comm_timing

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.ReLU(), torch.nn.Linear(64, 4))
    ddp = apex.parallel.DistributedDataParallel(model, message_size=200)
    assert len(ddp.buckets) > 1
    x = torch.randn(8, 16)
    ddp(x).sum().backward()  # first iteration: arrival-order rebucketing
    comm_timing.reset()
    comm_timing.enable(True)
    try:
        for _ in range(3):
            for p in model.parameters():
                p.grad = None
            ddp(x).sum().backward()
        pay = torch.arange(6, dtype=torch.float32) + rank
        g = _exchange_gather(pay, None)
        s = _exchange_sum(pay, None)
    finally:
        comm_timing.enable(False)
    assert comm_timing.count("allreduce_exposed") == 3
    assert comm_timing.count("bn_exchange") == 2
    per = comm_timing.summary(3)
    assert per["allreduce_exposed"] >= 0.0 and per["bn_exchange"] >= 0.0
    assert g.shape == (world, 6) and torch.equal(s.view(-1), pay * 0 + sum(torch.arange(6.0) + r for r in range(world)))
    # disabled: nothing recorded
    comm_timing.reset()
    ddp(x).sum().backward()
    assert comm_timing.count("allreduce_exposed") == 0
    dist.barrier()


def test_comm_timing_spans_ddp_and_bn_exchange():
    run_multiprocess(_worker, world=2)
