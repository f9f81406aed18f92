"""Multi-process (gloo, world_size 2) tests of the data-parallel layer (reference
tests/distributed/: DDP race-condition test, SyncBN two-GPU unit test, amp master params)."""
import pytest
import torch
import torch.distributed as dist

from tests._dist_utils import run_multiprocess


def _ddp_worker(rank, world, message_size, delay):
    import apex
    from apex.parallel import DistributedDataParallel as DDP

    torch.manual_seed(rank)  # different init per rank -> DDP must broadcast rank 0's
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    ddp = DDP(model, message_size=message_size, delay_allreduce=delay)
    w0 = [p.detach().clone() for p in model.parameters()]
    gathered = [torch.empty_like(w0[0]) for _ in range(world)]
    dist.all_gather(gathered, w0[0])
    assert torch.equal(gathered[0], gathered[1]), "params not broadcast"
    for it in range(3):
        for p in model.parameters():
            p.grad = None
        x = torch.full((2, 8), float(rank + 1 + it))
        ddp(x).sum().backward()
        # analytic check: grads equal the average of per-rank grads
        grads = [p.grad.detach().clone() for p in model.parameters()]
        # recompute per-rank grads without DDP
        ref_model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
        ref_model.load_state_dict(model.state_dict())
        per = []
        for r in range(world):
            ref_model.zero_grad()
            ref_model(torch.full((2, 8), float(r + 1 + it))).sum().backward()
            per.append([p.grad.clone() for p in ref_model.parameters()])
        for i, g in enumerate(grads):
            exp = sum(pr[i] for pr in per) / world
            torch.testing.assert_close(g, exp, rtol=1e-5, atol=1e-6)
    assert len(ddp.buckets) >= 1


@pytest.mark.parametrize("message_size,delay", [(1, False), (10000000, False), (40, True)])
def test_ddp_gloo(message_size, delay):
    run_multiprocess(_ddp_worker, 2, (message_size, delay))


def _syncbn_worker(rank, world, channel_last):
    import apex
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(0)
    full = torch.randn(8, 6, 5, 5, dtype=torch.float64).float()
    local = full[rank * 4:(rank + 1) * 4].clone().requires_grad_()
    bn = SyncBatchNorm(6, channel_last=channel_last)
    ref = torch.nn.BatchNorm2d(6)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, 6))
        bn.bias.copy_(torch.linspace(-1, 1, 6))
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    xin = local.permute(0, 2, 3, 1).contiguous() if channel_last else local
    y = bn(xin)
    y_nchw = y.permute(0, 3, 1, 2) if channel_last else y
    gy = torch.randn(8, 6, 5, 5, generator=torch.Generator().manual_seed(1))
    (y_nchw * gy[rank * 4:(rank + 1) * 4]).sum().backward()
    fr = full.clone().requires_grad_()
    yr = ref(fr)
    (yr * gy).sum().backward()
    torch.testing.assert_close(y_nchw, yr[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(local.grad, fr.grad[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-4)
    # weight grads are local sums (DDP averages them); compare the all-reduced sum
    gw = bn.weight.grad.clone()
    dist.all_reduce(gw)
    torch.testing.assert_close(gw, ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("channel_last", [False, True])
def test_syncbn_gloo(channel_last):
    run_multiprocess(_syncbn_worker, 2, (channel_last,))


def _convert_worker(rank, world):
    import apex
    from apex.models import resnet18

    m = apex.parallel.convert_syncbn_model(resnet18())
    n = sum(isinstance(x, apex.parallel.SyncBatchNorm) for x in m.modules())
    assert n == 20
    g = apex.parallel.create_syncbn_process_group(2)
    assert g is not None


def test_convert_syncbn_gloo():
    run_multiprocess(_convert_worker, 2, ())


# ------------------------------------------------------------------ DDP race condition
# (reference tests/distributed/DDP/ddp_race_condition_test.py: message_size=1 so every parameter
# is its own bucket, allreduce trigger params, 3 allreduce streams / communicators; the gradient
# sums are analytic, so any bucket fired before its gradient landed, or a stale buffer, shows up)
def _ddp_race_worker(rank, world, streams, trigger):
    from apex.parallel import DistributedDataParallel as DDP

    class Model(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.ones(4096))
            self.b = torch.nn.Parameter(torch.ones(4096))
            self.c = torch.nn.Parameter(torch.ones(2048))

        def forward(self, x):
            return (self.a * x).sum() + (self.b * x).sum() * 2.0 + (self.c * x[:2048]).sum() * 3.0

    model = Model()
    kw = dict(message_size=1, num_allreduce_streams=streams)
    if trigger:
        kw = dict(allreduce_trigger_params=[model.a, model.c], num_allreduce_streams=streams)
    ddp = DDP(model, **kw)
    for it in range(6):
        for p in model.parameters():
            p.grad = None
        x = torch.full((4096,), float((rank + 1) * (it + 1)))
        ddp(x).backward()
        mean_x = sum((r + 1) * (it + 1) for r in range(world)) / world
        assert torch.equal(model.a.grad, torch.full((4096,), mean_x)), (it, model.a.grad[:4])
        assert torch.equal(model.b.grad, torch.full((4096,), 2.0 * mean_x)), (it, model.b.grad[:4])
        assert torch.equal(model.c.grad, torch.full((2048,), 3.0 * mean_x)), (it, model.c.grad[:4])


@pytest.mark.parametrize("streams,trigger", [(3, False), (1, True), (2, True)])
def test_ddp_race_condition_gloo(streams, trigger):
    run_multiprocess(_ddp_race_worker, 2, (streams, trigger))


def test_ddp_race_condition_gloo_world8():
    """The 8-GPU node's rank count (bench.py --gpus 8 runs one DDP rank per GPU): bucket order,
    rank-0 rebucketing broadcast and the per-bucket all-reduces at world size 8."""
    run_multiprocess(_ddp_race_worker, 8, (1, False))


# ------------------------------------------------------------------ amp O2 master params across ranks
# (reference tests/distributed/amp_master_params: after DDP training with amp O2 the fp32 master
# params are identical on every rank and the low-precision model params are their casts)
def _amp_master_worker(rank, world):
    from apex import amp
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    torch.manual_seed(rank)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    opt = FusedAdam(model.parameters(), lr=1e-2)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    ddp = DDP(model)
    for it in range(4):
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(100 * rank + it))
        loss = ddp(x).float().pow(2).mean()
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
    masters = list(amp.master_params(opt))
    assert all(p.dtype == torch.float32 for p in masters)
    flat = torch.cat([p.detach().reshape(-1) for p in masters])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1]), "master params diverged across ranks"
    for m, p in zip(masters, model.parameters()):
        torch.testing.assert_close(p.detach().float(), m.detach().to(torch.bfloat16).float(), rtol=0, atol=0)


def test_amp_o2_master_params_equal_across_ranks_gloo():
    run_multiprocess(_amp_master_worker, 2, ())


# ------------------------------------------------------------------ SyncBN on a channels_last ResNet
# (round-1 bug: convert_syncbn_model(..., channel_last=True) on channels_last NCHW tensors read W as
# the channel dim; reference usage examples/imagenet/main_amp.py:118 passes channel_last this way)
def _syncbn_resnet_worker(rank, world, channel_last):
    import apex
    from apex.models import resnet18

    torch.manual_seed(0)
    base = resnet18(num_classes=10)
    ref = resnet18(num_classes=10)
    ref.load_state_dict(base.state_dict())
    model = apex.parallel.convert_syncbn_model(base, channel_last=channel_last).to(memory_format=torch.channels_last)
    full = torch.randn(4, 3, 32, 32, generator=torch.Generator().manual_seed(3))
    x = full[rank * 2:(rank + 1) * 2].contiguous(memory_format=torch.channels_last)
    out = model(x)
    out.sum().backward()
    ro = ref(full)
    ro.sum().backward()
    torch.testing.assert_close(out, ro[rank * 2:(rank + 1) * 2], rtol=2e-3, atol=2e-3)
    g = model.conv1.weight.grad.clone()
    dist.all_reduce(g)
    # fp32 sums over a different reduction order: compare relative to the gradient's scale
    scale = ref.conv1.weight.grad.abs().max().item()
    torch.testing.assert_close(g, ref.conv1.weight.grad, rtol=1e-2, atol=1e-2 * scale)
    for m, r in zip(model.modules(), ref.modules()):
        if isinstance(m, apex.parallel.SyncBatchNorm):
            torch.testing.assert_close(m.running_mean, r.running_mean, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("channel_last", [True, False])
def test_convert_syncbn_channels_last_resnet_fwd_bwd_gloo(channel_last):
    run_multiprocess(_syncbn_resnet_worker, 2, (channel_last,))


def _fused_bn_group_worker(rank, world):
    """The fused-BN ResNet with bn_group = world (bench.py --sync-bn): on CPU the group batch
    norm takes the SyncBatchNorm primitives; the result must equal the single-process model on
    the concatenated batch."""
    import apex
    from apex.models import resnet18

    torch.manual_seed(0)
    model = resnet18(num_classes=10, fused_bn=True, bn_group=world)
    ref = resnet18(num_classes=10)
    ref.load_state_dict(model.state_dict())
    full = torch.randn(4, 3, 32, 32, generator=torch.Generator().manual_seed(5))
    x = full[rank * 2:(rank + 1) * 2].contiguous(memory_format=torch.channels_last)
    model = model.to(memory_format=torch.channels_last)
    out = model(x)
    out.sum().backward()
    ro = ref(full)
    ro.sum().backward()
    torch.testing.assert_close(out, ro[rank * 2:(rank + 1) * 2], rtol=2e-3, atol=2e-3)
    g = model.conv1.weight.grad.clone()
    dist.all_reduce(g)
    scale = ref.conv1.weight.grad.abs().max().item()
    torch.testing.assert_close(g, ref.conv1.weight.grad, rtol=1e-2, atol=1e-2 * scale)
    # convert_syncbn_model keeps the fused modules (fused ReLU / residual inputs) and syncs them
    m2 = apex.parallel.convert_syncbn_model(resnet18(fused_bn=True))
    from apex.contrib.groupbn import BatchNorm2d_NHWC

    bns = [m for m in m2.modules() if isinstance(m, BatchNorm2d_NHWC)]
    assert bns and all(b.bn_group == world for b in bns)
    assert not any(isinstance(m, apex.parallel.SyncBatchNorm) for m in m2.modules())


def test_fused_resnet_bn_group_world_gloo():
    run_multiprocess(_fused_bn_group_worker, 2, ())


# ------------------------------------------------------------------ zero-copy DDP under fused amp
def _ddp_zero_copy_worker(rank, world):
    import os

    os.environ["APEX_AMD_AMP_SYNC_FREE"] = "force"
    from apex import amp
    from apex.amp._amp_state import _amp_state
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    _amp_state.sync_free_force = True
    torch.manual_seed(rank)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    opt = FusedAdam(model.parameters(), lr=1e-2, materialize_master_grads=False)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    assert _amp_state.sync_free, "fused (sync-free) amp path not active"
    ddp = DDP(model, message_size=1)  # one bucket per parameter
    params = list(model.parameters())
    copies = {"n": 0}
    orig_copy = torch.Tensor.copy_

    for it in range(5):
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(100 * rank + it))
        loss = ddp(x).float().pow(2).mean()
        opt.zero_grad()
        if it >= 2:
            # from the second step on every grad is its bucket view before backward ...
            for p in params:
                b, i = ddp._slot[id(p)]
                assert p.grad is not None and p.grad.data_ptr() == b.view_for(i).data_ptr(), it
        copies_before = ddp.grad_copies
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        if it >= 1:
            assert ddp.grad_copies == copies_before, (it, "per-parameter grad copies on the steady-state path")
        # ... and after it (autograd accumulated in place: the hook copied nothing)
        for p in params:
            b, i = ddp._slot[id(p)]
            lo = b.buffer.data_ptr()
            hi = lo + b.buffer.numel() * b.buffer.element_size()
            assert lo <= p.grad.data_ptr() < hi, (it, "grad outside its bucket")
        opt.step()
    masters = list(amp.master_params(opt))
    flat = torch.cat([p.detach().reshape(-1) for p in masters])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1]), "master params diverged across ranks"


def test_ddp_zero_copy_under_fused_amp_gloo():
    run_multiprocess(_ddp_zero_copy_worker, 2, ())


def _ddp_zero_copy_matches_reference_worker(rank, world):
    """Same training with DDP (zero-copy buckets) and with manual all-reduce of plain grads: the
    master weights must agree bit for bit."""
    import os

    os.environ["APEX_AMD_AMP_SYNC_FREE"] = "force"
    from apex import amp
    from apex.amp._amp_state import _amp_state
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    _amp_state.sync_free_force = True

    def make():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))

    def run(use_ddp):
        model = make()
        opt = FusedAdam(model.parameters(), lr=1e-2, materialize_master_grads=False)
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0,
                                    loss_scale=128.0)
        net = DDP(model) if use_ddp else model
        for it in range(4):
            x = torch.randn(8, 16, generator=torch.Generator().manual_seed(100 * rank + it))
            loss = net(x).float().pow(2).mean()
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as s:
                s.backward()
                if not use_ddp:
                    for p in model.parameters():
                        dist.all_reduce(p.grad)
                        p.grad.div_(world)
            opt.step()
        return torch.cat([p.detach().reshape(-1) for p in amp.master_params(opt)])

    a = run(True)
    b = run(False)
    torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_ddp_zero_copy_matches_manual_allreduce_gloo():
    # world 2 only: a bf16 sum of two values is order-independent, so the flat-bucket and the
    # per-tensor all-reduce agree bit for bit; at 8 ranks gloo's ring order differs between the two
    # and Adam amplifies the last-bit differences (world 8 is covered by the exact-sum race test)
    run_multiprocess(_ddp_zero_copy_matches_reference_worker, 2, ())


# ------------------------------------------------------- two amp optimizers over one DDP model
def _ddp_two_optimizers_worker(rank, world):
    import os

    os.environ["APEX_AMD_AMP_SYNC_FREE"] = "force"
    from apex import amp
    from apex.amp._amp_state import _amp_state
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    _amp_state.sync_free_force = True
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    first, second = list(model[0].parameters()), list(model[2].parameters())
    opt1 = FusedAdam(first, lr=1e-2, materialize_master_grads=False)
    opt2 = FusedAdam(second, lr=1e-2, materialize_master_grads=False)
    model, (opt1, opt2) = amp.initialize(model, [opt1, opt2], opt_level="O2", cast_model_type=torch.bfloat16,
                                         verbosity=0)
    ddp = DDP(model)  # default message size: ONE bucket shared by both optimizers' params
    assert len(ddp.buckets) == 1
    for it in range(3):
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(10 * rank + it))
        loss = ddp(x).float().pow(2).mean()
        opt1.zero_grad()
        opt2.zero_grad()
        with amp.scale_loss(loss, [opt1, opt2]) as s:
            s.backward()
        g2 = [p.grad.detach().clone() for p in model[2].parameters()]
        assert all(g.abs().sum() > 0 for g in g2), "second optimizer's grads are zero before any step"
        opt1.step()
        # opt1's post-step reset must not wipe the grads opt2 has not consumed yet
        for p, g in zip(model[2].parameters(), g2):
            assert p.grad is not None and torch.equal(p.grad, g), (it, "opt1.step() zeroed opt2's gradients")
        opt2.step()


def test_ddp_two_amp_optimizers_keep_each_others_grads_gloo():
    run_multiprocess(_ddp_two_optimizers_worker, 2, ())
