"""apex.transformer on CPU/gloo (model: reference tests/L0/run_transformer/run_{initialize,mappings,layers,
cross_entropy,random,data,pipeline_parallel}_test.py — those need >= 2 GPUs with NCCL; here the same
checks run as multi-process gloo tests so the distributed logic is covered in the CPU tier)."""
import pytest
import torch
import torch.distributed as dist

from tests._dist_utils import run_multiprocess


def test_topology_layout():
    from apex.transformer.parallel_state import ParallelTopology

    t = ParallelTopology(16, 2, 4)
    assert t.data_parallel_size == 2
    assert t.tensor_groups()[:2] == [[0, 1], [2, 3]]
    assert t.data_groups()[:4] == [[0, 2], [1, 3], [4, 6], [5, 7]]
    assert t.pipeline_groups()[:2] == [[0, 4, 8, 12], [1, 5, 9, 13]]
    for r in range(16):
        assert t.rank_of(*t.coords(r)) == r


def test_microbatch_calculators():
    from apex.transformer.microbatches import ConstantNumMicroBatches, RampupBatchsizeNumMicroBatches

    c = ConstantNumMicroBatches(64, 4, 2)
    assert c.get() == 8
    r = RampupBatchsizeNumMicroBatches(16, 16, 1000, 64, 4, 2)
    assert r.get() == 2
    r.update(1001, True)
    assert r.get() == 8


def test_batch_samplers_partition_dataset():
    from apex.transformer._data import MegatronPretrainingRandomSampler, MegatronPretrainingSampler

    seen = []
    for rank in range(2):
        s = MegatronPretrainingSampler(40, 0, 4, rank, 2)
        batches = list(s)
        assert all(len(b) == 4 for b in batches)
        seen += [i for b in batches for i in b]
    assert sorted(seen) == list(range(40))
    seen = []
    for rank in range(2):
        seen += [i for b in MegatronPretrainingRandomSampler(40, 0, 4, rank, 2) for i in b]
    assert sorted(seen) == list(range(40))


def _tp_worker(rank, world):
    from apex.transformer import parallel_state, tensor_parallel
    from apex.transformer.tensor_parallel import mappings

    parallel_state.initialize_model_parallel(world, 1)
    assert parallel_state.get_tensor_model_parallel_world_size() == world
    assert parallel_state.get_tensor_model_parallel_rank() == rank
    assert parallel_state.get_data_parallel_world_size() == 1
    tensor_parallel.model_parallel_cuda_manual_seed(1234)

    # mappings
    x = torch.arange(8, dtype=torch.float32).view(2, 4) + rank
    g = mappings._gather_along_last_dim(x)
    assert g.shape == (2, 4 * world)
    assert torch.equal(mappings._split_along_last_dim(g), x)
    x = torch.ones(3, requires_grad=True)
    y = tensor_parallel.copy_to_tensor_model_parallel_region(x)
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((3,), float(world)))
    s = mappings._reduce_scatter_along_first_dim(torch.ones(2 * world, 3) * (rank + 1))
    assert torch.equal(s, torch.full((2, 3), float(sum(range(1, world + 1)))))

    # column / row parallel vs the full linear (weights built from the same master)
    torch.manual_seed(0)
    inp, hid, out = 6, 8, 4
    col = tensor_parallel.ColumnParallelLinear(inp, hid, gather_output=False, keep_master_weight_for_test=True,
                                               use_cpu_initialization=True)
    row = tensor_parallel.RowParallelLinear(hid, out, input_is_parallel=True, keep_master_weight_for_test=True,
                                            use_cpu_initialization=True)
    with torch.no_grad():
        col.bias.copy_(torch.arange(col.bias.numel(), dtype=torch.float32) + rank * col.bias.numel())
        row.bias.fill_(0.5)
    xin = torch.randn(5, inp)
    dist.broadcast(xin, 0)
    h, _ = col(xin)
    y, _ = row(h)
    full_col_b = torch.arange(hid, dtype=torch.float32)
    ref = (xin @ col.master_weight.t() + full_col_b) @ row.master_weight.t() + 0.5
    torch.testing.assert_close(y, ref, atol=1e-5, rtol=1e-5)
    y.sum().backward()
    assert col.weight.grad.shape == col.weight.shape

    # vocab-parallel embedding + cross entropy vs torch
    vocab, dim = 16, 5
    emb = tensor_parallel.VocabParallelEmbedding(vocab, dim, use_cpu_initialization=True)
    ids = torch.tensor([[0, 3, 15, 8]])
    e = emb(ids)
    assert e.shape == (1, 4, dim)
    logits_full = torch.randn(3, 2, vocab)
    dist.broadcast(logits_full, 0)
    target = torch.randint(0, vocab, (3, 2))
    dist.broadcast(target, 0)
    part = vocab // world
    shard = logits_full[..., rank * part:(rank + 1) * part].clone().requires_grad_(True)
    loss = tensor_parallel.vocab_parallel_cross_entropy(shard, target)
    full = logits_full.clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(full.view(-1, vocab), target.view(-1), reduction="none").view(3, 2)
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)
    loss.sum().backward()
    ref.sum().backward()
    torch.testing.assert_close(shard.grad, full.grad[..., rank * part:(rank + 1) * part], atol=1e-5, rtol=1e-5)

    # broadcast_data
    data = {"a": torch.arange(6).view(2, 3), "b": torch.arange(4)} if rank == 0 else None
    out_d = tensor_parallel.broadcast_data(["a", "b"], data, torch.int64)
    assert torch.equal(out_d["a"], torch.arange(6).view(2, 3))

    # RNG tracker: TP stream differs per rank, default stream shared
    with tensor_parallel.get_cuda_rng_tracker().fork():
        r_tp = torch.rand(4)
    r_def = torch.rand(4)
    gathered = [torch.empty(4) for _ in range(world)]
    dist.all_gather(gathered, r_tp)
    assert not torch.equal(gathered[0], gathered[1])
    dist.all_gather(gathered, r_def)
    assert torch.equal(gathered[0], gathered[1])

    # checkpoint recompute reproduces dropout masks
    lin = torch.nn.Linear(4, 4)
    xx = torch.randn(3, 4, requires_grad=True)

    def f(t):
        with tensor_parallel.get_cuda_rng_tracker().fork():
            return torch.nn.functional.dropout(lin(t), 0.5, True)

    state = tensor_parallel.get_cuda_rng_tracker().get_states()
    cpu_state = torch.get_rng_state()
    out_ckpt = tensor_parallel.checkpoint(f, xx)
    out_ckpt.sum().backward()
    g1 = xx.grad.clone()
    tensor_parallel.get_cuda_rng_tracker().set_states(state)
    torch.set_rng_state(cpu_state)
    xx.grad = None
    f(xx).sum().backward()
    torch.testing.assert_close(g1, xx.grad)
    parallel_state.destroy_model_parallel()


def test_tensor_parallel_gloo_world2():
    run_multiprocess(_tp_worker, world=2)


def _pp_worker(rank, world, vpp):
    from apex.transformer import parallel_state
    from apex.transformer.pipeline_parallel import get_forward_backward_func, build_model
    from apex.transformer.pipeline_parallel.utils import setup_microbatch_calculator, destroy_microbatch_calculator

    parallel_state.initialize_model_parallel(1, world, vpp)
    num_mb, mbs, hidden = 4 if vpp is None else world * 2, 2, 8
    setup_microbatch_calculator(rank, None, num_mb * mbs, mbs, 1)
    nchunks = vpp or 1
    nstages = world * nchunks

    class Stage(torch.nn.Module):
        def __init__(self, pre_process, post_process):
            super().__init__()
            self.lin = torch.nn.Linear(hidden, hidden)
            self.input_tensor = None
            self.pre_process = pre_process

        def set_input_tensor(self, t):
            self.input_tensor = t

        def forward(self, x):
            inp = x if self.pre_process else self.input_tensor
            return torch.tanh(self.lin(inp))

    torch.manual_seed(0)
    all_layers = [torch.nn.Linear(hidden, hidden) for _ in range(nstages)]  # reference weights, same on all ranks

    def provider(pre_process, post_process):
        return Stage(pre_process, post_process)

    model = build_model(provider, wrap_with_ddp=False, virtual_pipeline_model_parallel_size=vpp)
    # stage (chunk c of rank r) holds layer c * world + r
    for c, m in enumerate(model):
        m.lin.load_state_dict(all_layers[c * world + rank].state_dict())

    torch.manual_seed(1)
    batch = [torch.randn(num_mb * mbs, hidden)]

    def fwd_step(mb, m):
        out = m(mb[0])

        def loss_fn(o):
            loss = (o ** 2).mean()
            return loss, loss.detach()

        return out, loss_fn

    fb = get_forward_backward_func(vpp, world)
    losses = fb(fwd_step, batch, model if vpp else model[0], forward_only=False, tensor_shape=(mbs, hidden),
                dtype=torch.float32)

    # sequential reference
    ref_layers = [torch.nn.Linear(hidden, hidden) for _ in range(nstages)]
    for l, r in zip(ref_layers, all_layers):
        l.load_state_dict(r.state_dict())
    ref_losses = []
    for k in range(num_mb):
        x = batch[0][k * mbs:(k + 1) * mbs]
        for l in ref_layers:
            x = torch.tanh(l(x))
        loss = (x ** 2).mean() / num_mb
        loss.backward()
        ref_losses.append(loss.detach() * num_mb)
    if parallel_state.is_pipeline_last_stage(ignore_virtual=True):
        torch.testing.assert_close(torch.stack(losses), torch.stack(ref_losses), atol=1e-6, rtol=1e-5)
    for c, m in enumerate(model):
        ref = ref_layers[c * world + rank]
        torch.testing.assert_close(m.lin.weight.grad, ref.weight.grad, atol=1e-6, rtol=1e-5)
    destroy_microbatch_calculator()
    parallel_state.destroy_model_parallel()


def test_pipeline_1f1b_gloo_world2():
    run_multiprocess(_pp_worker, world=2, args=(None,))


def test_pipeline_1f1b_gloo_world4():
    run_multiprocess(_pp_worker, world=4, args=(None,))


def test_pipeline_interleaved_gloo_world4():
    run_multiprocess(_pp_worker, world=4, args=(2,))


def _no_pipe_worker(rank, world):
    from apex.transformer import parallel_state
    from apex.transformer.pipeline_parallel import get_forward_backward_func
    from apex.transformer.pipeline_parallel.utils import setup_microbatch_calculator, destroy_microbatch_calculator

    parallel_state.initialize_model_parallel(1, 1)
    setup_microbatch_calculator(rank, None, 8, 2, world)
    torch.manual_seed(0)
    model = torch.nn.Linear(4, 1)
    fb = get_forward_backward_func(None, 1)
    batch = [torch.randn(4, 4)]

    def fwd_step(mb, m):
        out = m(mb[0])
        return out, lambda o: ((o ** 2).mean(), (o ** 2).mean().detach())

    losses = fb(fwd_step, batch, model, forward_only=False)
    assert len(losses) == 2
    destroy_microbatch_calculator()
    parallel_state.destroy_model_parallel()


def test_no_pipelining_gloo():
    run_multiprocess(_no_pipe_worker, world=2)


def test_bias_dropout_add_mask_statistics_and_checkpoint_restore():
    """Counter-hash dropout: keep rate matches p, masks are a pure function of (seed, offset),
    and activation checkpointing restores the counter streams so a recompute redraws them."""
    from apex.transformer.functional.fused_bias_dropout_add import fused_bias_dropout_add, keep_mask
    from apex.transformer.tensor_parallel import get_counter_rng_streams

    keep = keep_mask(5, 11, 1 << 20, 0.1)
    assert abs(keep.float().mean().item() - 0.9) < 2e-3
    assert torch.equal(keep, keep_mask(5, 11, 1 << 20, 0.1))
    assert not torch.equal(keep, keep_mask(5, 12, 1 << 20, 0.1))
    x, r, b = torch.randn(64, 32), torch.randn(64, 32), torch.randn(32)
    y = fused_bias_dropout_add(x, b, r, 0.1, True, 5, 11)
    k = keep_mask(5, 11, x.numel(), 0.1).view(x.shape)
    torch.testing.assert_close(y, r + torch.where(k, (x + b) / 0.9, torch.zeros_like(x)))
    torch.testing.assert_close(fused_bias_dropout_add(x, b, r, 0.1, False, 5, 11), r + (x + b))
    st = get_counter_rng_streams()
    saved = st.get_states()
    a = st.next("hidden_dropout")
    st.set_states(saved)
    assert st.next("hidden_dropout") == a
