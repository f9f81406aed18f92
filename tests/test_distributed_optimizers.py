"""ZeRO distributed optimizers and legacy contrib optimizers.

Model: reference apex/contrib/test/optimizers/test_dist_adam.py (DistributedFusedAdam on every
rank vs torch.optim.AdamW on the full model with all-reduced gradients, params compared after
several steps) and test_distributed_fused_lamb.py (LAMB vs reference LAMB math).  CPU tiers run
world_size 2 over gloo (fp32 params, so the comparison is tight)."""
import copy
import sys

import pytest
import torch
import torch.distributed as dist

from tests._dist_utils import run_multiprocess


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(13, 37), torch.nn.Tanh(), torch.nn.Linear(37, 29),
                               torch.nn.Tanh(), torch.nn.Linear(29, 5))


def _batches(rank, n=4):
    g = torch.Generator().manual_seed(100 + rank)
    return [(torch.randn(8, 13, generator=g), torch.randn(8, 5, generator=g)) for _ in range(n)]


def _ref_lamb_step(params, grads, state, lr, b1, b2, eps, wd, step, grad_averaging=True):
    for p, g in zip(params, grads):
        st = state.setdefault(id(p), {"m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        st["m"].mul_(b1).add_(g, alpha=(1 - b1) if grad_averaging else 1.0)
        st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
        mh = st["m"] / (1 - b1 ** step)
        vh = st["v"] / (1 - b2 ** step)
        u = mh / (vh.sqrt() + eps) + wd * p
        pn, un = p.norm(), u.norm()
        ratio = (pn / un) if (pn > 0 and un > 0) else 1.0
        p.sub_(lr * ratio * u)


def _worker(rank, world, kind, num_blocks, max_grad_norm, extra=None):
    from apex.contrib.optimizers import DistributedFusedAdam, DistributedFusedAdamV3, DistributedFusedLAMB

    model = _model()
    ref = copy.deepcopy(model)
    kw = dict(lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.01, dwu_num_blocks=num_blocks,
              min_block_elems=256)
    kw.update(extra or {})
    if kind == "adam":
        opt = DistributedFusedAdam(model.parameters(), max_grad_norm=max_grad_norm, **kw)
        ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.01)
    elif kind == "adam_v3":
        opt = DistributedFusedAdamV3(model.parameters(), max_grad_norm=max_grad_norm, **kw)
        assert opt._flat.mode == "ar"
        ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.01)
        ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.01)
    else:
        if kind == "lamb_noavg":
            kw["grad_averaging"] = False
        opt = DistributedFusedLAMB(model.parameters(), max_grad_norm=max_grad_norm, **kw)
        ref_state = {}
    assert opt._flat.num_blocks >= 1
    for step, (x, y) in enumerate(_batches(rank), start=1):
        loss = torch.nn.functional.mse_loss(model(x), y)
        loss.backward()
        opt.step()
        # reference: full model, gradient averaged over ranks
        ref.zero_grad()
        torch.nn.functional.mse_loss(ref(x), y).backward()
        grads = []
        for p in ref.parameters():
            dist.all_reduce(p.grad)
            p.grad.div_(world)
            grads.append(p.grad)
        if max_grad_norm > 0:
            torch.nn.utils.clip_grad_norm_(list(ref.parameters()), max_grad_norm)
        if kind in ("adam", "adam_v3"):
            ref_opt.step()
        else:
            with torch.no_grad():
                _ref_lamb_step(list(ref.parameters()), [p.grad for p in ref.parameters()], ref_state, 1e-2, 0.9, 0.99,
                               1e-8, 0.01, step, grad_averaging=(kind != "lamb_noavg"))
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p, q, atol=2e-5, rtol=1e-4)
        if max_grad_norm > 0:
            assert opt.L2_grad_norm is not None
    # model params are views into the flat buffer; grads were zeroed into the buffer
    assert all(p.grad is not None and float(p.grad.abs().sum()) == 0 for p in model.parameters())
    if (extra or {}).get("dwu_group_size"):
        g = extra["dwu_group_size"]
        assert opt._flat.world == g and opt._flat.ar_world == world // g and opt._flat.dp_size == world
        # replicas in different groups hold identical parameters
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        parts = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(parts, flat)
        for q in parts[1:]:
            torch.testing.assert_close(q, parts[0], rtol=0, atol=0)


@pytest.mark.parametrize("kind", ["adam", "lamb", "lamb_noavg"])
@pytest.mark.parametrize("num_blocks,max_grad_norm", [(1, 0.0), (3, 0.0), (2, 0.05)])
def test_distributed_optimizer_matches_full_model(kind, num_blocks, max_grad_norm):
    run_multiprocess(_worker, world=2, args=(kind, num_blocks, max_grad_norm))


@pytest.mark.parametrize("kind", ["adam", "lamb", "adam_v3"])
@pytest.mark.parametrize("extra", [dict(dwu_group_size=2), dict(dwu_group_size=2, reduce_dtype=torch.float64),
                                   dict(dwu_group_size=2, predivide=False)])
def test_distributed_optimizer_two_level_world4(kind, extra):
    """world 4 sharded over groups of 2 (reference dwu_group_size): reduce-scatter inside the group
    plus all-reduce across groups must train exactly like the full model on the global batch."""
    run_multiprocess(_worker, world=4, args=(kind, 2, 0.05 if kind == "lamb" else 0.0, extra))


@pytest.mark.parametrize("num_blocks", [1, 3])
def test_distributed_adam_v3_allreduce_mode(num_blocks):
    run_multiprocess(_worker, world=2, args=("adam_v3", num_blocks, 0.0))


def _overflow_worker(rank, world):
    from apex.contrib.optimizers import DistributedFusedAdam

    model = _model(1)
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, min_block_elems=128)
    before = [p.detach().clone() for p in model.parameters()]
    x, y = _batches(rank, 1)[0]
    xb = x.clone()
    if rank == 1:  # non-finite grads on one rank (reduced during backward) skip the step on every rank
        xb[0, 0] = float("inf")
    torch.nn.functional.mse_loss(model(xb), y).backward()
    opt.step()
    assert opt.has_overflow
    for p, b in zip(model.parameters(), before):
        assert torch.equal(p, b)
    # next, clean step proceeds; step counter only advanced once
    torch.nn.functional.mse_loss(model(x), y).backward()
    opt.step()
    assert not opt.has_overflow
    assert float(opt._step_t) == 1.0
    # sharded checkpoint round trip
    sd = opt.state_dict()
    opt2 = DistributedFusedAdam(_model(1).parameters(), lr=1e-2, min_block_elems=128)
    opt2.load_state_dict(sd)
    torch.testing.assert_close(opt2._m, opt._m)
    torch.testing.assert_close(opt2._flat.flat_param, opt._flat.flat_param)


def test_distributed_adam_overflow_skip_and_checkpoint():
    run_multiprocess(_overflow_worker, world=2)


def _gathered_master(opt):
    """The full fp32 master vector in flat-buffer layout (every rank's shards)."""
    flat = opt._flat
    parts = [torch.empty_like(flat.master) for _ in range(flat.world)]
    dist.all_gather(parts, flat.master.contiguous())
    rows = []
    for b in range(flat.num_blocks):
        rows += [parts[r][b] for r in range(flat.world)]
    return torch.cat(rows)


def _fp8_worker(rank, world, kind, fp8):
    from apex.contrib.optimizers import DistributedFusedAdam, DistributedFusedLAMB

    model = _model(3)
    plain = copy.deepcopy(model)
    cls = DistributedFusedAdam if kind == "adam" else DistributedFusedLAMB
    kw = dict(lr=1e-2, weight_decay=0.01, dwu_num_blocks=2, min_block_elems=256)
    if fp8 == "e5m2":
        opt = cls(model.parameters(), e5m2_allgather=True, **kw)
    else:
        opt = cls(model.parameters(), allgather_dtype=torch.float8_e4m3fn, **kw)
    ref_opt = cls(plain.parameters(), **kw)
    dt = torch.float8_e5m2 if fp8 == "e5m2" else torch.float8_e4m3fn
    for x, y in _batches(rank, 3):
        for m, o in ((model, opt), (plain, ref_opt)):
            torch.nn.functional.mse_loss(m(x), y).backward()
            o.step()
        # every rank (the owner included) holds exactly the fp8-rounded master
        master = _gathered_master(opt)
        flat = opt._flat.flat_param
        for p, off in zip(opt._flat.params, opt._flat.offsets):
            n = p.numel()
            want = master[off:off + n].to(dt).to(p.dtype)
            assert torch.equal(p.detach().reshape(-1), want)
        # and stays close to uncompressed training (fp8 rounding of the weights only)
        for p, q in zip(model.parameters(), plain.parameters()):
            tol = 0.13 if fp8 == "e5m2" else 0.07
            torch.testing.assert_close(p, q, rtol=tol, atol=0.03)
    parts = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(parts, flat)
    assert all(torch.equal(parts[0], q) for q in parts[1:])


@pytest.mark.parametrize("kind", ["adam", "lamb"])
@pytest.mark.parametrize("fp8", ["e5m2", "e4m3"])
def test_distributed_fp8_allgather(kind, fp8):
    run_multiprocess(_fp8_worker, world=2, args=(kind, fp8))


def _revert_worker(rank, world, wd_mode):
    from apex.contrib.optimizers import DistributedFusedAdamV2

    model = _model(4)
    opt = DistributedFusedAdamV2(model.parameters(), lr=1e-2, weight_decay=0.05, min_block_elems=256,
                                 dwu_num_blocks=2, adam_w_mode=(wd_mode == "adamw"))
    b = _batches(rank, 3)
    for x, y in b[:2]:
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
    snap = dict(master=opt._flat.master.clone(), m=opt._m.clone(), v=opt._v.clone(), step=opt._step_t.clone(),
                params=[p.detach().clone() for p in model.parameters()])
    x, y = b[2]
    torch.nn.functional.mse_loss(model(x), y).backward()
    opt.step()
    assert not torch.equal(opt._flat.master, snap["master"])
    opt.revert_step()
    torch.testing.assert_close(opt._flat.master, snap["master"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(opt._m, snap["m"], rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(opt._v, snap["v"], rtol=1e-3, atol=1e-9)
    assert torch.equal(opt._step_t, snap["step"])
    for p, q in zip(model.parameters(), snap["params"]):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-7)
    with pytest.raises(RuntimeError):
        opt.revert_step()  # one step back only
    # redoing the step lands where the first attempt did
    torch.nn.functional.mse_loss(model(x), y).backward()
    opt.step()
    torch.nn.functional.mse_loss(model(x), y).backward()  # a later backward invalidates the revert
    with pytest.raises(RuntimeError):
        opt.revert_step()


@pytest.mark.parametrize("wd_mode", ["adamw", "l2"])
def test_distributed_adam_revert_step_without_clones(wd_mode):
    run_multiprocess(_revert_worker, world=2, args=(wd_mode,))


def _accum_worker(rank, world):
    from apex.contrib.optimizers import DistributedFusedAdam

    model = _model(2)
    ref = copy.deepcopy(model)
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, weight_decay=0.0, min_block_elems=128)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    b = _batches(rank, 2)
    opt.set_is_accumulation_step(True)
    torch.nn.functional.mse_loss(model(b[0][0]), b[0][1]).backward()
    opt.set_is_accumulation_step(False)
    model.zero_grad(set_to_none=False)  # drop the accumulated micro-batch (zeroes the flat buffer in place)
    torch.nn.functional.mse_loss(model(b[0][0]), b[0][1]).backward()
    torch.nn.functional.mse_loss(model(b[1][0]), b[1][1]).backward()  # second micro-batch, hooks re-fire
    opt.step()
    for x, y in b:
        torch.nn.functional.mse_loss(ref(x), y).backward()
    for p in ref.parameters():
        dist.all_reduce(p.grad)
        p.grad.div_(world)
    ref_opt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, atol=2e-5, rtol=1e-4)


def test_distributed_adam_accumulation_and_refire():
    run_multiprocess(_accum_worker, world=2)


def test_distributed_adam_single_process_set_to_none():
    """world=1 without init: grads re-adopted after zero_grad(set_to_none=True)."""
    from apex.contrib.optimizers import DistributedFusedAdam

    model = _model(3)
    ref = copy.deepcopy(model)
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, weight_decay=0.0)
    ref_opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    for x, y in _batches(0, 3):
        model.zero_grad(set_to_none=True)
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
        ref_opt.zero_grad()
        torch.nn.functional.mse_loss(ref(x), y).backward()
        ref_opt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, atol=2e-5, rtol=1e-4)


def test_contrib_legacy_optimizers_with_fp16_optimizer():
    from apex.contrib.optimizers import FP16_Optimizer, FusedAdam, FusedLAMB, FusedSGD

    torch.manual_seed(0)
    for cls, kw, ref_cls, ref_kw in [
        (FusedAdam, dict(lr=1e-2), torch.optim.AdamW, dict(lr=1e-2, weight_decay=0.0)),
        (FusedSGD, dict(lr=0.1, momentum=0.9), torch.optim.SGD, dict(lr=0.1, momentum=0.9)),
    ]:
        model = _model(4)
        ref = copy.deepcopy(model)
        opt = FP16_Optimizer(cls(model.parameters(), **kw), static_loss_scale=128.0)
        ref_opt = ref_cls(ref.parameters(), **ref_kw)
        for x, y in _batches(0, 3):
            opt.zero_grad()
            opt.backward(torch.nn.functional.mse_loss(model(x), y))
            opt.step()
            ref_opt.zero_grad()
            torch.nn.functional.mse_loss(ref(x), y).backward()
            ref_opt.step()
        for p, q in zip(model.parameters(), ref.parameters()):
            torch.testing.assert_close(p, q, atol=1e-4, rtol=1e-3)
    model = _model(5)
    ref = copy.deepcopy(model)
    opt = FusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1e9, betas=(0.9, 0.99), eps=1e-8)
    st = {}
    for step, (x, y) in enumerate(_batches(0, 3), start=1):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
        for p in ref.parameters():
            p.grad = None
        torch.nn.functional.mse_loss(ref(x), y).backward()
        with torch.no_grad():
            _ref_lamb_step(list(ref.parameters()), [p.grad for p in ref.parameters()], st, 1e-2, 0.9, 0.99, 1e-8,
                           0.01, step)
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, atol=1e-5, rtol=1e-4)


def _lamb_overflow_worker(rank, world):
    """DistributedFusedLAMB's step is gated on the device skip flag (no host read of it): an
    overflow on one rank leaves every rank's weights and moments untouched and does not advance
    the device step count; the sharded checkpoint carries that count."""
    from apex.contrib.optimizers import DistributedFusedLAMB

    model = _model(2)
    opt = DistributedFusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, min_block_elems=128)
    before = [p.detach().clone() for p in model.parameters()]
    x, y = _batches(rank, 1)[0]
    xb = x.clone()
    if rank == 1:
        xb[0, 0] = float("inf")
    torch.nn.functional.mse_loss(model(xb), y).backward()
    opt.step()
    assert opt.has_overflow
    for p, b in zip(model.parameters(), before):
        assert torch.equal(p, b)
    assert float(opt._m.abs().sum()) == 0 and float(opt._step_t) == 0.0
    torch.nn.functional.mse_loss(model(x), y).backward()
    opt.step()
    assert not opt.has_overflow and float(opt._step_t) == 1.0
    assert any(not torch.equal(p, b) for p, b in zip(model.parameters(), before))
    sd = opt.state_dict()
    opt2 = DistributedFusedLAMB(_model(2).parameters(), lr=1e-2, weight_decay=0.01, min_block_elems=128)
    opt2.load_state_dict(sd)
    assert float(opt2._step_t) == 1.0
    torch.testing.assert_close(opt2._v, opt._v)


def test_distributed_lamb_overflow_skip_on_device():
    run_multiprocess(_lamb_overflow_worker, world=2)


def _lamb_sync_free_worker(rank, world):
    from apex.contrib.optimizers import DistributedFusedLAMB

    dev = torch.device("cuda", 0)
    model = _model(4).to(dev)
    opt = DistributedFusedLAMB(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0,
                               min_block_elems=128)
    x, y = (t.to(dev) for t in _batches(rank, 1)[0])

    def one():
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()

    one()
    one()  # work tables / buffers built
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        one()
        one()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert float(opt._step_t) == 4.0


@pytest.mark.gpu
def test_gpu_distributed_lamb_step_makes_no_host_sync():
    """The whole LAMB step (unscale / overflow check / grad-norm clip, stage 1, the fused
    [2, num_params] norm all-reduce, stage 2, all-gather) runs under torch's sync debug mode set
    to raise on any device -> host synchronization."""
    run_multiprocess(_lamb_sync_free_worker, world=1, backend="nccl")


def _fp8_overflow_worker(rank, world, kind):
    """fp8 all-gather + an overflow on the very first step: the skipped step still gathers the
    payload (the skip flag stays on the device), which must hold the current master weights —
    not the zeros it was allocated with — and, after a checkpoint load, the loaded weights."""
    from apex.contrib.optimizers import DistributedFusedAdam, DistributedFusedLAMB

    cls = DistributedFusedAdam if kind == "adam" else DistributedFusedLAMB
    kw = dict(lr=1e-2, weight_decay=0.01, dwu_num_blocks=2, min_block_elems=256, e5m2_allgather=True)
    dt = torch.float8_e5m2
    model = _model(6)
    before = [p.detach().clone() for p in model.parameters()]
    opt = cls(model.parameters(), **kw)
    x, y = _batches(rank, 1)[0]
    xb = x.clone()
    if rank == 1:
        xb[0, 0] = float("inf")
    torch.nn.functional.mse_loss(model(xb), y).backward()
    opt.step()
    assert opt.has_overflow
    for p, b in zip(model.parameters(), before):
        # the weights went through the fp8 gather unchanged (rounded), not zeroed
        assert torch.equal(p.detach(), b.to(dt).to(b.dtype))
        assert float(p.detach().abs().sum()) > 0
    torch.nn.functional.mse_loss(model(x), y).backward()
    opt.step()
    assert not opt.has_overflow
    sd = opt.state_dict()
    trained = [p.detach().clone() for p in model.parameters()]
    # a fresh optimizer over different weights: load, then overflow on its first step
    model2 = _model(7)
    opt2 = cls(model2.parameters(), **kw)
    opt2.load_state_dict(sd)
    torch.nn.functional.mse_loss(model2(xb), y).backward()
    opt2.step()
    assert opt2.has_overflow
    master = _gathered_master(opt2)
    for p, q, off in zip(model2.parameters(), trained, opt2._flat.offsets):
        n = p.numel()
        assert torch.equal(p.detach().reshape(-1), master[off:off + n].to(dt).to(p.dtype))
        torch.testing.assert_close(p.detach(), q, rtol=0.13, atol=0.03)


@pytest.mark.parametrize("kind", ["adam", "lamb"])
def test_distributed_fp8_allgather_overflow_on_first_step(kind):
    run_multiprocess(_fp8_overflow_worker, world=2, args=(kind,))


class _NoHostRead:
    """Raise on any host read of a tensor's value (``item`` / ``bool`` / ``float`` / ``int`` /
    ``tolist`` / ``numpy``) inside the block: the CPU stand-in for torch's CUDA sync debug mode,
    which only sees device syncs."""

    _NAMES = ("item", "__bool__", "__float__", "__int__", "__index__", "tolist", "numpy")

    def __enter__(self):
        self._saved = {n: getattr(torch.Tensor, n) for n in self._NAMES}

        saved = self._saved

        def boom(name):
            def f(*a, **k):
                # the CPU stand-ins of the device kernels (ops/multi_tensor_ref.py) compute on the
                # host by construction; only the optimizer's own Python path is checked
                fr = sys._getframe(1)
                while fr is not None:
                    if fr.f_code.co_filename.endswith("multi_tensor_ref.py"):
                        return saved[name](*a, **k)
                    fr = fr.f_back
                raise AssertionError(f"host read of a tensor value ({name}) inside the step")
            return f

        for n in self._NAMES:
            setattr(torch.Tensor, n, boom(n))
        return self

    def __exit__(self, *exc):
        for n, f in self._saved.items():
            setattr(torch.Tensor, n, f)
        return False


def _sync_free_cpu_worker(rank, world, kind, ag):
    from apex.contrib.optimizers import DistributedFusedAdam, DistributedFusedLAMB

    cls = DistributedFusedAdam if kind == "adam" else DistributedFusedLAMB
    model = _model(4)
    opt = cls(model.parameters(), lr=1e-2, weight_decay=0.01, max_grad_norm=1.0, min_block_elems=128,
              dwu_num_blocks=2, e5m2_allgather=ag)
    batches = _batches(rank, 4)
    for i, (x, y) in enumerate(batches):
        xb = x.clone()
        if i == 2 and rank == 0:
            xb[0, 0] = float("nan")  # one overflow step, gated on the device flag
        torch.nn.functional.mse_loss(model(xb), y).backward()
        if i == 0:
            opt.step()  # first step builds the buffers
            continue
        with _NoHostRead():
            opt.step()
    assert float(opt._step_t) == 3.0


@pytest.mark.parametrize("kind", ["adam", "lamb"])
@pytest.mark.parametrize("ag", [False, True])
def test_distributed_step_reads_no_host_value_world2(kind, ag):
    """world 2 (gloo): the whole sharded step — overflow flag all-reduce, grad-norm clip, the LAMB
    [2, num_params] norm all-reduce, stages 1/2, the (fp8) all-gather — never reads a tensor value
    on the host, overflow step included (the GPU tier checks the same under sync debug mode)."""
    run_multiprocess(_sync_free_cpu_worker, world=2, args=(kind, ag))
