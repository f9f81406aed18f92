"""hipBLASLt plan picks made rank-consistent (fused_dense.sync_lt_plans): the per-process timed
choice is recorded as an index into the support-screened candidate list and rank 0's table is
broadcast and applied on every rank of the group."""
import pytest
import torch

from tests._dist_utils import run_multiprocess


def _worker(rank, world):
    import torch.distributed as dist

    from apex import _native
    from apex.fused_dense import fused_dense as fd

    lt = _native.submodule("lt_gemm")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(4096, 1024, device=dev, dtype=torch.bfloat16)
    w = torch.randn(3072, 1024, device=dev, dtype=torch.bfloat16)
    b = torch.randn(3072, device=dev, dtype=torch.bfloat16)
    lt.clear_cache()
    y = lt.linear(x, w, b, lt.EPI_BIAS)[0]
    table = lt.plan_choices()
    assert len(table) == 1 and table[0][10] >= 1
    key = list(table[0])
    # force a different local pick on rank 1, then sync: every rank ends with rank 0's pick
    if rank == 1 and key[10] > 1:
        key2 = key[:11] + [(key[11] + 1) % key[10]]
        assert lt.set_plan_choice(key2, 0)
    n = fd.sync_lt_plans(None)
    assert n == 1
    picks = [None] * world
    dist.all_gather_object(picks, lt.plan_choices()[0][11])
    assert len(set(picks)) == 1, picks
    # the synced pick computes the same product
    y2 = lt.linear(x, w, b, lt.EPI_BIAS)[0]
    torch.testing.assert_close(y2.float(), (x.float() @ w.float().t() + b.float()), atol=0.5, rtol=2e-2)
    # a key this process never planned is refused, as is an out-of-range pick
    assert not lt.set_plan_choice([1, 2, 3, 1, 1, 1, 0, 0, key[8], key[9], 1, 0], 0)
    assert not lt.set_plan_choice(key[:11] + [key[10]], 0)
    del y


@pytest.mark.gpu
def test_gpu_lt_plan_picks_synced_across_ranks():
    # two ranks sharing the one GPU over gloo (the broadcast is of host objects)
    run_multiprocess(_worker, world=2, backend="gloo")


def test_sync_lt_plans_noop_without_group():
    from apex.fused_dense import sync_lt_plans

    assert sync_lt_plans(None) == 0


class _FakeLt:
    """Stand-in for the hipBLASLt wrapper's plan table (CPU tier)."""

    def __init__(self, rank):
        self.rank, self.picks = rank, {}

    def plan_choices(self):
        return [k + (v,) for k, v in sorted(self.picks.items())]

    def set_plan_choice(self, key, dev):
        self.picks[tuple(key[:-1])] = key[-1]
        return True


def _decision_worker(rank, world):
    """The sync decision follows the TP problem sequence (identical on every rank), not the
    process-wide plan table: rank 1 planning extra library GEMMs of its own (a non-TP layer) must
    neither make it enter a broadcast alone nor skip one the other rank enters."""
    import torch.distributed as dist

    from apex import _native
    from apex.fused_dense import fused_dense as fd

    fake = _FakeLt(rank)
    orig = _native.submodule
    _native.submodule = lambda name: fake if name == "lt_gemm" else orig(name)
    try:
        fake.picks[("fwd", 64, 32, 16)] = rank  # rank-local timed picks differ
        if rank == 1:
            fake.picks[("other", 1, 2, 3)] = 7  # a non-TP problem planned on rank 1 only
        assert fd.maybe_sync_lt_plans(None, ("fwd", 64, 32, 16))
        assert fake.picks[("fwd", 64, 32, 16)] == 0  # rank 0's pick everywhere
        if rank == 1:
            fake.picks[("other2", 4, 5, 6)] = 3
        assert not fd.maybe_sync_lt_plans(None, ("fwd", 64, 32, 16))  # same problem: no collective
        assert fd.maybe_sync_lt_plans(None, ("wgrad", 64, 32, 16))
        dist.barrier()
    finally:
        _native.submodule = orig


def test_lt_sync_decision_is_rank_consistent():
    run_multiprocess(_decision_worker, world=2)
