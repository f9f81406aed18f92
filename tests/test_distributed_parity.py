"""Distributed test parity with the reference's multi-process suites, run over gloo on CPU:

* SyncBatchNorm with a different batch size per rank
  (reference tests/distributed/synced_batchnorm/two_gpu_test_different_batch_size.py),
* SyncBatchNorm inside process groups (test_groups.py) and the fused NHWC BN with
  ``bn_group`` and unequal per-rank batches,
* tensor-parallel layers under autocast, with and without sequence parallelism and the async
  grad all-reduce, against the unsharded model (tests/L0/run_transformer/run_layers_test.py),
* the model-parallel RNG tracker (run_random_test.py),
* the pipeline schedules with a ramped global batch size (run_dynamic_batchsize_test.py)."""
import pytest
import torch
import torch.distributed as dist

from tests._dist_utils import run_multiprocess


# ================================================================== SyncBN, unequal batches
def _bn_ref(full, w, b):
    ref = torch.nn.BatchNorm2d(full.size(1), momentum=0.1)
    with torch.no_grad():
        ref.weight.copy_(w)
        ref.bias.copy_(b)
    return ref


def _syncbn_uneven_worker(rank, world, channel_last):
    from apex.parallel import SyncBatchNorm

    sizes = [6, 2, 5, 3][:world]
    torch.manual_seed(2809)
    full = torch.randn(sum(sizes), 4, 5, 5) * 50.0
    gy_full = torch.randint(0, 10, full.shape).float() / 10.0
    lo = sum(sizes[:rank])
    local = full[lo:lo + sizes[rank]].clone().requires_grad_()
    w, b = torch.linspace(0.5, 1.5, 4), torch.linspace(-1, 1, 4)
    bn = SyncBatchNorm(4, channel_last=channel_last)
    with torch.no_grad():
        bn.weight.copy_(w)
        bn.bias.copy_(b)
    xin = local.permute(0, 2, 3, 1).contiguous() if channel_last else local
    y = bn(xin)
    y = y.permute(0, 3, 1, 2) if channel_last else y
    (y * gy_full[lo:lo + sizes[rank]]).sum().backward()
    ref = _bn_ref(full, w, b)
    fr = full.clone().requires_grad_()
    yr = ref(fr)
    (yr * gy_full).sum().backward()
    torch.testing.assert_close(y, yr[lo:lo + sizes[rank]], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(local.grad, fr.grad[lo:lo + sizes[rank]], rtol=1e-4, atol=1e-4)
    for mine, theirs in ((bn.weight.grad, ref.weight.grad), (bn.bias.grad, ref.bias.grad)):
        g = mine.clone()
        dist.all_reduce(g)
        torch.testing.assert_close(g, theirs, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("channel_last", [False, True])
def test_syncbn_different_batch_size_per_rank_gloo(channel_last):
    run_multiprocess(_syncbn_uneven_worker, 2, (channel_last,))


def _syncbn_groups_worker(rank, world):
    import apex
    from apex.parallel import SyncBatchNorm

    group = apex.parallel.create_syncbn_process_group(2)  # ranks {0,1} and {2,3}
    torch.manual_seed(7)
    data = torch.randn(world, 3, 4, 6, 6)  # one 3-sample batch per rank
    w, b = torch.linspace(0.5, 1.5, 4), torch.linspace(-1, 1, 4)
    bn = SyncBatchNorm(4, process_group=group)
    with torch.no_grad():
        bn.weight.copy_(w)
        bn.bias.copy_(b)
    x = data[rank].clone().requires_grad_()
    y = bn(x)
    y.sum().backward()
    g0 = (rank // 2) * 2
    full = torch.cat([data[g0], data[g0 + 1]]).requires_grad_()
    ref = _bn_ref(full, w, b)
    yr = ref(full)
    yr.sum().backward()
    i = rank - g0
    torch.testing.assert_close(y, yr[3 * i:3 * i + 3], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad, full.grad[3 * i:3 * i + 3], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    # groups are independent: the other group's statistics differ
    rm = [torch.empty(4) for _ in range(world)]
    dist.all_gather(rm, bn.running_mean.contiguous())
    assert torch.equal(rm[0], rm[1]) and torch.equal(rm[2], rm[3]) and not torch.equal(rm[0], rm[2])


def test_syncbn_process_groups_world4_gloo():
    run_multiprocess(_syncbn_groups_worker, 4, ())


def _fused_bn_group_uneven_worker(rank, world):
    from apex.contrib.groupbn import BatchNorm2d_NHWC

    sizes = [5, 2]
    torch.manual_seed(11)
    full = torch.randn(sum(sizes), 8, 4, 4) * 3 + 1
    lo = sum(sizes[:rank])
    x = full[lo:lo + sizes[rank]].clone().to(memory_format=torch.channels_last).requires_grad_()
    bn = BatchNorm2d_NHWC(8, fuse_relu=True, bn_group=world, torch_channels_last=True)
    y = bn(x)
    gy = torch.linspace(-1, 1, y.numel()).view_as(y)
    (y * gy[:]).sum().backward()
    ref = torch.nn.BatchNorm2d(8)
    fr = full.clone().requires_grad_()
    yr = torch.relu(ref(fr))
    gfull = torch.cat([torch.linspace(-1, 1, s * 8 * 16).view(s, 8, 4, 4) for s in sizes])
    (yr * gfull).sum().backward()
    torch.testing.assert_close(y, yr[lo:lo + sizes[rank]], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad, fr.grad[lo:lo + sizes[rank]], rtol=1e-4, atol=1e-4)


def test_fused_nhwc_bn_group_uneven_batches_gloo():
    run_multiprocess(_fused_bn_group_uneven_worker, 2, ())


# ================================================================== tensor-parallel layers
def _layers_worker(rank, world, sequence_parallel, autocast):
    from apex.transformer import parallel_state, tensor_parallel
    from apex.transformer.tensor_parallel import mappings

    parallel_state.initialize_model_parallel(world, 1)
    tensor_parallel.model_parallel_cuda_manual_seed(99)
    torch.manual_seed(5)
    seq, batch, hid, ffn = 8, 3, 16, 32
    col = tensor_parallel.ColumnParallelLinear(hid, ffn, gather_output=False, keep_master_weight_for_test=True,
                                               use_cpu_initialization=True,
                                               sequence_parallel_enabled=sequence_parallel)
    row = tensor_parallel.RowParallelLinear(ffn, hid, input_is_parallel=True, keep_master_weight_for_test=True,
                                            use_cpu_initialization=True,
                                            sequence_parallel_enabled=sequence_parallel)
    x_full = torch.randn(seq, batch, hid)
    dist.broadcast(x_full, 0)
    gy_full = torch.randn(seq, batch, hid)
    dist.broadcast(gy_full, 0)
    # full-width reference from the master weights and the gathered column bias
    cb = [torch.empty_like(col.bias) for _ in range(world)]
    dist.all_gather(cb, col.bias.detach().contiguous())
    wc = col.master_weight.clone().requires_grad_()
    wr = row.master_weight.clone().requires_grad_()
    bc = torch.cat(cb).requires_grad_()
    br = row.bias.detach().clone().requires_grad_()
    xr = x_full.clone().requires_grad_()
    ctx = torch.autocast("cpu", dtype=torch.bfloat16) if autocast else torch.autocast("cpu", enabled=False)
    with ctx:
        ref = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(xr, wc, bc)), wr, br)
    ref.float().backward(gy_full)

    if sequence_parallel:  # activations enter and leave 1/tp along the sequence
        chunk = seq // world
        x = x_full[rank * chunk:(rank + 1) * chunk].clone().requires_grad_()
        gy = gy_full[rank * chunk:(rank + 1) * chunk]
    else:
        x, gy = x_full.clone().requires_grad_(), gy_full
    with ctx:
        h, _ = col(x)
        y, _ = row(torch.nn.functional.gelu(h))
    y.float().backward(gy)
    tol = dict(rtol=3e-2, atol=3e-2) if autocast else dict(rtol=1e-5, atol=1e-5)
    want = ref[rank * chunk:(rank + 1) * chunk] if sequence_parallel else ref
    torch.testing.assert_close(y.float(), want.float(), **tol)
    want_dx = xr.grad[rank * chunk:(rank + 1) * chunk] if sequence_parallel else xr.grad
    torch.testing.assert_close(x.grad, want_dx, **tol)
    part = ffn // world
    torch.testing.assert_close(col.weight.grad, wc.grad[rank * part:(rank + 1) * part], **tol)
    torch.testing.assert_close(row.weight.grad, wr.grad[:, rank * part:(rank + 1) * part], **tol)
    torch.testing.assert_close(col.bias.grad, bc.grad[rank * part:(rank + 1) * part], **tol)
    if sequence_parallel:  # the replicated row bias sees only this rank's sequence slice
        g = row.bias.grad.clone()
        dist.all_reduce(g)
        torch.testing.assert_close(g, br.grad, **tol)
    else:
        torch.testing.assert_close(row.bias.grad, br.grad, **tol)
    assert mappings is not None
    parallel_state.destroy_model_parallel()


@pytest.mark.parametrize("sequence_parallel", [False, True])
@pytest.mark.parametrize("autocast", [False, True])
def test_tensor_parallel_layers_vs_full_model_gloo(sequence_parallel, autocast):
    run_multiprocess(_layers_worker, 2, (sequence_parallel, autocast))


# ================================================================== RNG tracker
def _random_worker(rank, world):
    from apex.transformer import parallel_state, tensor_parallel
    from apex.transformer.tensor_parallel import random as tp_random

    parallel_state.initialize_model_parallel(world, 1)
    tensor_parallel.model_parallel_cuda_manual_seed(123)
    tracker = tensor_parallel.get_cuda_rng_tracker()
    states = tracker.get_states()
    assert tp_random._MODEL_PARALLEL_RNG_TRACKER_NAME in states
    with tracker.fork():
        a = torch.rand(16)
    with tracker.fork():
        b = torch.rand(16)
    assert not torch.equal(a, b)  # the stream advances
    tracker.set_states(states)
    with tracker.fork():
        a2 = torch.rand(16)
    assert torch.equal(a, a2)  # restored
    parts = [torch.empty(16) for _ in range(world)]
    dist.all_gather(parts, a)
    assert not torch.equal(parts[0], parts[1])  # model-parallel streams differ across TP ranks
    with pytest.raises(Exception):
        tracker.add(tp_random._MODEL_PARALLEL_RNG_TRACKER_NAME, 1)  # duplicate name
    with pytest.raises(Exception):
        with tracker.fork("no-such-stream"):
            pass
    tracker.reset()
    assert tracker.get_states() == {}
    parallel_state.destroy_model_parallel()


def test_model_parallel_rng_tracker_gloo():
    run_multiprocess(_random_worker, 2, ())


# ================================================================== dynamic batch size
def _dynamic_bs_worker(rank, world):
    from apex.transformer import parallel_state
    from apex.transformer.pipeline_parallel import get_forward_backward_func
    from apex.transformer.pipeline_parallel.utils import (destroy_microbatch_calculator, get_num_microbatches,
                                                          setup_microbatch_calculator, update_num_microbatches)

    parallel_state.initialize_model_parallel(1, 1)
    micro, gbs = 2, 16
    # ramp the global batch from 4 to 16 in steps of 4 over 48 samples (data-parallel size `world`)
    setup_microbatch_calculator(rank, [4, 4, 48], gbs, micro, world)
    torch.manual_seed(0)
    model = torch.nn.Linear(4, 1)
    ref = torch.nn.Linear(4, 1)
    ref.load_state_dict(model.state_dict())
    fb = get_forward_backward_func(None, 1)
    consumed, seen = 0, []
    g = torch.Generator().manual_seed(rank)
    while consumed < 96:
        update_num_microbatches(consumed)
        n_mb = get_num_microbatches()
        seen.append(n_mb)
        batch = [torch.randn(n_mb * micro, 4, generator=g)]

        def fwd_step(mb, m):
            out = m(mb[0])
            return out, lambda o: ((o ** 2).mean(), (o ** 2).mean().detach())  # the schedule divides by n_mb

        model.zero_grad()
        losses = fb(fwd_step, batch, model, forward_only=False)
        assert len(losses) == n_mb
        ref.zero_grad()
        for k in range(n_mb):
            (ref(batch[0][k * micro:(k + 1) * micro]) ** 2).mean().div(n_mb).backward()
        torch.testing.assert_close(model.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-6)
        consumed += n_mb * micro * world
    assert seen[0] == 1 and seen[-1] == gbs // (micro * world) and sorted(seen) == seen
    destroy_microbatch_calculator()
    parallel_state.destroy_model_parallel()


def test_dynamic_batch_size_pipeline_schedule_gloo():
    run_multiprocess(_dynamic_bs_worker, 2, ())
