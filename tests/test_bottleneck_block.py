"""The fused training bottleneck node (ops/bottleneck_bn.py: BN statistics in the 1x1 conv
epilogues, bn2 apply+ReLU as conv3's operand prologue, one gradient out) against the fp32
PyTorch bottleneck with the same weights: forward output, input gradient, every weight / BN
parameter gradient and the running statistics."""
import copy
import statistics

import pytest
import torch

CASES = [
    # inplanes, planes, stride, downsample, h, batch
    (256, 64, 1, False, 14, 3),    # identity block (stage-1 widths)
    (64, 64, 1, True, 14, 2),      # first block of stage 1: stride-1 1x1 downsample
    (256, 128, 2, True, 16, 2),    # first block of stage 2: stride-2 downsample
    (512, 128, 1, False, 7, 4),    # identity, conv1 K = 512
    (1024, 256, 1, False, 7, 2),   # identity, conv1 K = 1024 (library fallback forward)
]


def _make(inplanes, planes, stride, downsample, fused):
    from apex.models.resnet import Bottleneck, conv1x1, _fused_bn
    import torch.nn as nn

    ds = None
    if downsample:
        bn = _fused_bn(planes * 4, False) if fused else nn.BatchNorm2d(planes * 4)
        ds = nn.Sequential(conv1x1(inplanes, planes * 4, stride, native=fused), bn)
    return Bottleneck(inplanes, planes, stride, ds, fused_bn=fused)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize("inplanes,planes,stride,downsample,h,batch", CASES)
@pytest.mark.parametrize("block_node", [True, False])
def test_gpu_fused_bottleneck_matches_fp32(inplanes, planes, stride, downsample, h, batch, block_node):
    import apex  # noqa: F401
    from apex.ops import bottleneck_bn

    torch.manual_seed(0)
    ref = _make(inplanes, planes, stride, downsample, fused=False).cuda().float()
    for m in ref.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
            m.running_mean.uniform_(-0.1, 0.1)
    blk = _make(inplanes, planes, stride, downsample, fused=True).cuda()
    blk.load_state_dict(ref.state_dict())
    # amp O2 layout: bf16 convs, fp32 BN params, channels_last
    for mod in blk.modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.to(torch.bfloat16)
    blk = blk.to(memory_format=torch.channels_last)
    blk.train()
    ref.train()

    x = torch.randn(batch, inplanes, h, h, device="cuda")
    xb = x.to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_(True)
    xr = xb.detach().float().requires_grad_(True)
    assert bottleneck_bn.block_supported(blk, xb)
    old_enabled = bottleneck_bn._ENABLED
    bottleneck_bn._ENABLED = block_node
    calls = {"n": 0}
    orig = bottleneck_bn._BottleneckFn.forward

    def counted(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    bottleneck_bn._BottleneckFn.forward = staticmethod(counted)
    try:
        y = blk(xb)
    finally:
        bottleneck_bn._BottleneckFn.forward = staticmethod(orig)
        bottleneck_bn._ENABLED = old_enabled
    assert calls["n"] == int(block_node) and not isinstance(y, tuple)
    yr = ref(xr)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, yr) < 2e-2, _rel(y, yr)

    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16).to(memory_format=torch.channels_last))
    yr.backward(gy)
    pairs = dict(ref.named_parameters())
    errs = {"x": _rel(xb.grad, xr.grad)}
    for name, p in blk.named_parameters():
        assert p.grad is not None, name
        errs[name] = _rel(p.grad, pairs[name].grad)
    print("rel errors", {k: round(v, 4) for k, v in errs.items()})
    # bf16 activations / gradients through three batch norms at a few thousand pixels: ~5-10 %
    # relative error against fp32 for BOTH fused paths (the per-module path measures the same)
    assert max(errs.values()) < 0.15, errs
    bufs = dict(ref.named_buffers())
    for name, b in blk.named_buffers():
        if name.endswith("running_mean") or name.endswith("running_var"):
            torch.testing.assert_close(b, bufs[name], atol=2e-3, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("inplanes,planes,stride,downsample,h,batch", CASES)
def test_gpu_fused_bottleneck_node_vs_module_path(inplanes, planes, stride, downsample, h, batch):
    """The block node against the per-module fused path on identical bf16 inputs: the two
    differ only in rounding order, so they agree far more closely than either does with fp32."""
    import apex  # noqa: F401
    from apex.ops import bottleneck_bn

    torch.manual_seed(1)
    a = _make(inplanes, planes, stride, downsample, fused=True).cuda()
    for mod in a.modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.to(torch.bfloat16)
    a = a.to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(batch, inplanes, h, h, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = None
    outs = []
    for mod, node in ((a, True), (b, False)):
        xi = x.clone().requires_grad_(True)
        old = bottleneck_bn._ENABLED
        bottleneck_bn._ENABLED = node
        try:
            y = mod(xi)
            if gy is None:
                gy = torch.randn_like(y)
            y.backward(gy)
        finally:
            bottleneck_bn._ENABLED = old
        outs.append((y.detach(), xi.grad, {n: p.grad for n, p in mod.named_parameters()}))
    (ya, ga, pa), (yb, gb, pb) = outs
    assert _rel(ya, yb) < 1e-2
    assert _rel(ga, gb) < 6e-2, _rel(ga, gb)
    for n in pa:
        assert _rel(pa[n], pb[n]) < 8e-2, (n, _rel(pa[n], pb[n]))


@pytest.mark.gpu
@pytest.mark.parametrize("force_native", [False, True])
def test_gpu_fused_bottleneck_resnet50_step_matches_module_path(force_native, monkeypatch):
    """A full fused-BN ResNet-50 training step, chained block nodes (BlockLink hand-offs) vs the
    per-module fused path (APEX_AMD_FUSED_BLOCK off), both against an fp32 PyTorch ResNet-50
    with the same weights.  Through 16 bf16 residual blocks at random init the per-parameter
    gradients of BOTH bf16 paths sit far from fp32 (median relative error ~1.2, dominated by
    bf16 rounding amplified by the batch-norm backward — tools/dbg_block_chain.py), so the check
    is statistical: the node path must not be less accurate than the module path.
    force_native: every native 1x1 route (incl. the masked dgrad + reduction hand-off across
    blocks) even at this small size."""
    import statistics

    import apex  # noqa: F401
    from apex.models import resnet50
    from apex.ops import bottleneck_bn

    monkeypatch.setattr(bottleneck_bn, "FORCE_NATIVE", force_native)
    calls = {"red": 0}
    conv = apex._native.require("conv").conv
    orig = conv.dgrad_bnred

    class _Spy:
        def __getattr__(self, name):
            if name == "dgrad_bnred":
                def f(*a, **k):
                    calls["red"] += a[3] is not None  # the cross-block (ReLU bits) hand-offs
                    return orig(*a, **k)
                return f
            return getattr(conv, name)

    monkeypatch.setattr(bottleneck_bn, "_conv", lambda: _Spy())
    torch.manual_seed(0)
    ref = resnet50().cuda()
    m1 = resnet50(fused_bn=True).cuda()
    m1.load_state_dict(ref.state_dict())
    m1 = m1.to(memory_format=torch.channels_last)
    for mod in m1.modules():
        if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear)):
            mod.to(torch.bfloat16)
    m2 = copy.deepcopy(m1)
    x = torch.randn(32, 3, 96, 96, device="cuda")
    tgt = torch.randint(0, 1000, (32,), device="cuda")
    l0 = torch.nn.functional.cross_entropy(ref(x), tgt)
    l0.backward()
    xb = x.to(torch.bfloat16).to(memory_format=torch.channels_last)

    def step(model, enabled):
        old = bottleneck_bn._ENABLED
        bottleneck_bn._ENABLED = enabled
        try:
            loss = torch.nn.functional.cross_entropy(model(xb).float(), tgt)
            loss.backward()
        finally:
            bottleneck_bn._ENABLED = old
        return loss.detach()

    l1, l2 = step(m1, True), step(m2, False)
    torch.testing.assert_close(l1, l0.detach(), atol=5e-2, rtol=1e-2)
    torch.testing.assert_close(l2, l0.detach(), atol=5e-2, rtol=1e-2)
    # 16 bottlenecks, 15 boundaries; the masked-dgrad hand-off where the route takes it
    assert calls["red"] == (15 if force_native else 0), calls
    g0, g2 = dict(ref.named_parameters()), dict(m2.named_parameters())
    e1 = [_rel(p.grad, g0[n].grad) for n, p in m1.named_parameters()]
    e2 = [_rel(g2[n].grad, g0[n].grad) for n, _ in m1.named_parameters()]
    assert statistics.median(e1) <= 1.1 * statistics.median(e2) + 0.02, (statistics.median(e1), statistics.median(e2))
    # the classifier sits above every block: compare the two paths there directly
    fc1, fc2 = _rel(m1.fc.weight.grad, g0["fc.weight"].grad), _rel(m2.fc.weight.grad, g0["fc.weight"].grad)
    assert fc1 <= 1.5 * fc2 + 0.02, (fc1, fc2)


def _chain(bn_group=1, peer=True, dtype=torch.bfloat16):
    """A 3-block stage-1 chain (downsampling block + 2 identity blocks), fused BN, 16-bit convs."""
    import torch.nn as nn

    from apex.contrib.groupbn import BatchNorm2d_NHWC
    from apex.models.resnet import Bottleneck, conv1x1

    ds = nn.Sequential(conv1x1(64, 256, 1, native=True),
                       BatchNorm2d_NHWC(256, fuse_relu=False, torch_channels_last=True))
    blocks = [Bottleneck(64, 64, 1, ds, fused_bn=True), Bottleneck(256, 64, fused_bn=True),
              Bottleneck(256, 64, fused_bn=True)]
    for b in blocks[:-1]:
        b.fork_out = True
    chain = nn.ModuleList(blocks)
    for m in chain.modules():
        if isinstance(m, nn.Conv2d):
            m.to(dtype)
        if isinstance(m, BatchNorm2d_NHWC):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    return chain


def _run_chain(chain, x, gy, node, bn_group=1, group=None, peer=True, linked=True):
    import apex  # noqa: F401
    from apex.contrib.groupbn import BatchNorm2d_NHWC
    from apex.models.resnet import run_linked
    from apex.ops import bottleneck_bn

    if bn_group > 1:
        for m in chain.modules():
            if isinstance(m, BatchNorm2d_NHWC):
                m.synchronize_over(group, peer_memory=peer)
    calls = {"n": 0, "red": 0}
    orig, conv = bottleneck_bn._BottleneckFn.forward, bottleneck_bn._conv()
    orig_red = conv.dgrad_bnred

    class _Spy:
        def __getattr__(self, name):
            if name == "dgrad_bnred":
                def f(*a, **k):
                    calls["red"] += a[3] is not None
                    return orig_red(*a, **k)
                return f
            return getattr(conv, name)

    def counted(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    old = bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE, bottleneck_bn._conv
    bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE = node, True
    bottleneck_bn._conv = lambda: _Spy()
    bottleneck_bn._BottleneckFn.forward = staticmethod(counted)
    d0 = bottleneck_bn.DEFERRED_TAKEN[0]
    try:
        xi = x.clone().requires_grad_(True)
        if linked:
            y = run_linked(list(chain), xi)
        else:
            y = xi
            for blk in chain:
                y = blk(y)
        if isinstance(y, tuple):
            y = y[0]
        y.backward(gy)
    finally:
        bottleneck_bn._BottleneckFn.forward = staticmethod(orig)
        bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE, bottleneck_bn._conv = old
    calls["deferred"] = bottleneck_bn.DEFERRED_TAKEN[0] - d0
    return y.detach(), xi.grad, {n: p.grad for n, p in chain.named_parameters()}, calls


@pytest.mark.gpu
def test_gpu_bottleneck_chain_linked_vs_unlinked():
    """a 3-block chain with every native route forced.  The linked walk
    (BlockLink: block i+1's conv1 dgrad masks with block i's ReLU bits and does its bn3 backward
    reduction) against the same nodes called one by one (no hand-off): the forward is identical
    and the backward differs only in the order of one reduction's sums, so a wrong hand-off
    (mask, reduction, coefficients) shows as an O(1) difference while the correct one agrees to
    rounding.  Against fp32 all three bf16 arms (linked, unlinked, per-module) sit at the same
    ~18 % dx / ~17 % median parameter-gradient distance through 3 blocks (tools/dbg_chain_link.py,
    profiles/chain_link_r04.jsonl), so the per-module path is checked at that noise level only."""
    torch.manual_seed(3)
    a = _chain().cuda().to(memory_format=torch.channels_last).train()
    b, c = copy.deepcopy(a), copy.deepcopy(a)
    x = torch.randn(4, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    ya, ga, pa, ca = _run_chain(a, x, gy, True)
    yb, gb, pb, cb = _run_chain(b, x, gy, True, linked=False)
    yc, gc, pc, cc = _run_chain(c, x, gy, False)
    assert ca["n"] == 3 and cb["n"] == 3 and cc["n"] == 0, (ca, cb, cc)
    # the linked walk computes blocks 1 and 2's outputs in the next block's conv1 (deferred output
    # pass); the unlinked arm runs every output pass itself
    assert ca["deferred"] == 2 and cb["deferred"] == 0, (ca, cb)
    assert ca["red"] == 2 and cb["red"] == 0, (ca, cb)  # both boundaries took the hand-off when linked
    assert torch.equal(ya, yb)
    assert _rel(ga, gb) < 2e-2, _rel(ga, gb)
    for n in pa:
        assert _rel(pa[n], pb[n]) < 2e-2, (n, _rel(pa[n], pb[n]))
    assert _rel(ya, yc) < 1e-2
    assert _rel(ga, gc) < 0.3, _rel(ga, gc)
    for n in pa:
        assert _rel(pa[n], pc[n]) < 0.35, (n, _rel(pa[n], pc[n]))
    for (n, ba), bb in zip(a.named_buffers(), c.buffers()):
        if n.endswith("running_mean") or n.endswith("running_var"):
            torch.testing.assert_close(ba, bb, atol=2e-3, rtol=2e-2)


def _sync_chain_worker(rank, world, peer):
    """bn_group = 2 over 2 ranks sharing the GPU (gloo + peer memory or host staging): each rank
    runs the 3-block node chain on half of the batch; every BN's statistics and backward sums are
    exchanged, so rank r reproduces slice r of the 1-rank full-batch node chain."""
    import torch.distributed as dist

    torch.cuda.set_device(0)
    torch.manual_seed(3)
    full = _chain().cuda().to(memory_format=torch.channels_last).train()
    mine = copy.deepcopy(full)
    x = torch.randn(8, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = torch.randn(8, 256, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    yf, gf, pf, _ = _run_chain(full, x, gy, True)
    sl = slice(rank * 4, rank * 4 + 4)
    ys, gs, ps, calls = _run_chain(mine, x[sl].contiguous(memory_format=torch.channels_last),
                                   gy[sl].contiguous(memory_format=torch.channels_last), True, world, None, peer)
    assert calls["n"] == 3, calls
    # the statistics are the full batch's up to summation order (merged Welford payloads vs one
    # shifted sum), which flips bf16 roundings and grows to a few % through 3 blocks' BN backward
    # (measured 6-7 % dx; all bf16 arms are ~18 % from fp32, profiles/chain_link_r04.jsonl); a
    # wrong exchange (local count, missing sums) is an O(1) error
    assert _rel(ys, yf[sl]) < 1e-2, _rel(ys, yf[sl])
    assert _rel(gs, gf[sl]) < 0.15, _rel(gs, gf[sl])
    for n, g in ps.items():
        tot = g.detach().float().cpu()
        dist.all_reduce(tot)  # local parameter gradients: the group sum is the full-batch gradient
        assert _rel(tot, pf[n].cpu()) < 0.15, (n, _rel(tot, pf[n].cpu()))
    for (n, bs), bf in zip(mine.named_buffers(), full.buffers()):
        if n.endswith("running_mean") or n.endswith("running_var"):
            torch.testing.assert_close(bs, bf, atol=2e-3, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("peer", [True, False])
def test_gpu_bottleneck_chain_syncbn_two_ranks(peer):
    """the fused node under SyncBN (bn_group = 2) matches the full-batch node."""
    from tests._dist_utils import run_multiprocess

    run_multiprocess(_sync_chain_worker, 2, (peer,), timeout=180)


def _sync_resnet_worker(rank, world):
    """ResNet-50 with bn_group = world (what ``bench.py --sync-bn`` builds): all 16 bottlenecks
    stay fused nodes with the statistics synchronized, and one training step runs."""
    import apex  # noqa: F401
    from apex.models import resnet50
    from apex.ops import bottleneck_bn

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    model = resnet50(fused_bn=True, bn_group=world).cuda().to(memory_format=torch.channels_last)
    for m in model.modules():
        if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear)):
            m.to(torch.bfloat16)
    x = torch.randn(4, 3, 64, 64, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    tgt = torch.randint(0, 1000, (4,), device="cuda")
    n0 = bottleneck_bn.NODE_CALLS[0]
    loss = torch.nn.functional.cross_entropy(model(x).float(), tgt)
    assert bottleneck_bn.NODE_CALLS[0] - n0 == 16, bottleneck_bn.NODE_CALLS[0] - n0
    loss.backward()
    assert torch.isfinite(loss).item()
    assert all(torch.isfinite(p.grad).all() for p in model.parameters() if p.grad is not None)


@pytest.mark.gpu
def test_gpu_resnet50_syncbn_keeps_the_16_nodes():
    from tests._dist_utils import run_multiprocess

    run_multiprocess(_sync_resnet_worker, 2, (), timeout=180)


def _chain_f64_reference(chain, x, gy):
    """The chain's module path in float64 on the CPU (the groupbn modules run their torch
    reference there): output, input gradient and parameter gradients."""
    ref = copy.deepcopy(chain).cpu().double().train()
    xi = x.detach().cpu().double().requires_grad_(True)
    y = xi
    for blk in ref:
        y = blk(y)
    if isinstance(y, tuple):
        y = y[0]
    y.backward(gy.detach().cpu().double())
    return y.detach(), xi.grad, {n: p.grad for n, p in ref.named_parameters()}


def _arm_distances(dtype, seed=3):
    torch.manual_seed(seed)
    base = _chain(dtype=dtype).cuda().to(memory_format=torch.channels_last).train()
    x = torch.randn(4, 64, 14, 14, device="cuda").to(dtype).to(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 14, 14, device="cuda").to(dtype).to(memory_format=torch.channels_last)
    y64, g64, p64 = _chain_f64_reference(base, x, gy)
    out = {}
    for arm, node, linked in (("linked", True, True), ("unlinked", True, False), ("module", False, True)):
        c = copy.deepcopy(base)
        y, g, pg, _ = _run_chain(c, x, gy, node, linked=linked)
        out[arm] = dict(y=y, g=g, p=pg,
                        dy=_rel(y.cpu().double(), y64), dg=_rel(g.cpu().double(), g64),
                        dp=statistics.median(_rel(pg[n].cpu().double(), p64[n]) for n in p64))
    return out


@pytest.mark.gpu
def test_gpu_bottleneck_chain_fp16_arm_pins_the_tolerances():
    """the chain tolerances above (0.3 dx / 0.35 params vs the per-module
    path) are set by bf16 rounding noise; an O(0.1) bug in a hand-off would hide under them.  With
    fp16 operands (3 more mantissa bits) every arm's distance to a float64 reference must shrink
    by >= 2.5x — a real bug does not shrink with precision — and the node arms (linked, unlinked) must
    stay as close to float64 as the per-module path (within 2x)."""
    bf, hf = _arm_distances(torch.bfloat16), _arm_distances(torch.float16)
    for prec, d in (("bf16", bf), ("fp16", hf)):
        print(prec, {a: {k: round(d[a][k], 5) for k in ("dy", "dg", "dp")} for a in d})
    # measured (r05, 1 x MI355X): every arm shrinks 3-4x from bf16 to fp16 (BN backward's mean
    # subtraction amplifies the activations' rounding, so not the full 8x of 3 mantissa bits); a
    # wrong hand-off or coefficient would leave an O(0.1) distance that does not shrink at all
    for arm in ("linked", "unlinked", "module"):
        for k in ("dy", "dg", "dp"):
            assert hf[arm][k] * 2.5 <= bf[arm][k] + 1e-4, (arm, k, bf[arm][k], hf[arm][k])
    for k in ("dg", "dp"):
        assert hf["linked"][k] <= 2 * hf["module"][k] + 1e-3, (k, hf["linked"][k], hf["module"][k])
        assert hf["unlinked"][k] <= 2 * hf["module"][k] + 1e-3, (k, hf["unlinked"][k], hf["module"][k])
    # the fp16 node arms against each other: only one reduction's summation order differs
    assert _rel(hf["linked"]["g"], hf["unlinked"]["g"]) < 5e-3


def _sync_chain_fp16_worker(rank, world):
    """The 2-rank SyncBN chain with fp16 convs: its distance to the 1-rank full-batch node chain
    shrinks with precision like every other arm (an exchange bug would not)."""
    torch.cuda.set_device(0)
    res = {}
    for dt in (torch.bfloat16, torch.float16):
        torch.manual_seed(3)
        full = _chain(dtype=dt).cuda().to(memory_format=torch.channels_last).train()
        mine = copy.deepcopy(full)
        x = torch.randn(8, 64, 14, 14, device="cuda").to(dt).to(memory_format=torch.channels_last)
        gy = torch.randn(8, 256, 14, 14, device="cuda").to(dt).to(memory_format=torch.channels_last)
        yf, gf, _, _ = _run_chain(full, x, gy, True)
        sl = slice(rank * 4, rank * 4 + 4)
        ys, gs, _, _ = _run_chain(mine, x[sl].contiguous(memory_format=torch.channels_last),
                                  gy[sl].contiguous(memory_format=torch.channels_last), True, world, None, True)
        res[dt] = (_rel(ys, yf[sl]), _rel(gs, gf[sl]))
    print(rank, res)
    # measured: 0.074-0.076 (bf16) -> 0.019-0.020 (fp16), 3.7-3.9x; an exchange bug (local count,
    # missing sums) would not shrink
    assert res[torch.float16][1] * 2.5 <= res[torch.bfloat16][1] + 1e-4, res
    assert res[torch.float16][1] < 0.03, res


@pytest.mark.gpu
def test_gpu_bottleneck_chain_syncbn_fp16_arm():
    from tests._dist_utils import run_multiprocess

    run_multiprocess(_sync_chain_fp16_worker, 2, (), timeout=240)


@pytest.mark.gpu
@pytest.mark.parametrize("inplanes,planes,stride,h,batch", [(64, 64, 1, 14, 2), (256, 128, 2, 16, 2)])
def test_gpu_downsample_dx_prologue_matches_apply_pass(inplanes, planes, stride, h, batch, monkeypatch):
    """The downsample BN's dx computed as the downsample dgrad's operand prologue (kProBnBwd,
    ``_DS_DX_PRO``) against the reduction + dx pass + plain dgrad: the prologue runs the dx pass's
    arithmetic, so the dx it writes for the weight gradient — and with it every gradient of the
    block — is bitwise the same."""
    import apex  # noqa: F401
    from apex.ops import bottleneck_bn

    torch.manual_seed(3)
    a = _make(inplanes, planes, stride, True, fused=True).cuda()
    for mod in a.modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.to(torch.bfloat16)
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
    a = a.to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(batch, inplanes, h, h, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = None
    outs = []
    for mod, pro in ((a, True), (b, False)):
        monkeypatch.setattr(bottleneck_bn, "_DS_DX_PRO", pro)
        xi = x.clone().requires_grad_(True)
        y = mod(xi)
        if gy is None:
            gy = torch.randn_like(y)
        y.backward(gy)
        outs.append((y.detach(), xi.grad, {n: p.grad for n, p in mod.named_parameters()}))
    (ya, ga, pa), (yb, gb, pb) = outs
    assert torch.equal(ya, yb)
    # the downsample branch is bitwise (its dx, written by the prologue, is the dx pass's value);
    # elsewhere the stride-2 block runs library 3x3 gradients whose summation order may vary from
    # call to call (MIOpen weight gradient), so those compare at rounding level
    for n in pa:
        if n.startswith("downsample"):
            assert torch.equal(pa[n], pb[n]), (n, _rel(pa[n], pb[n]))
        else:
            assert _rel(pa[n], pb[n]) < 1e-3, (n, _rel(pa[n], pb[n]))
    if stride == 1:
        assert torch.equal(ga, gb), _rel(ga, gb)
    else:
        assert _rel(ga, gb) < 1e-3, _rel(ga, gb)


@pytest.mark.gpu
def test_gpu_chain_downsample_reduction_in_block_above(monkeypatch):
    """The downsampling block's downsample-BN backward reduction accumulated by the block above's
    conv1 dgrad epilogue (BlockLink.yd, ``_DS_RED``: part [4, G, C]) against the reduction pass
    over dm and yd: the same sums in another order, so the arms agree to rounding and a wrong
    operand / mean / slab shows as an O(1) difference."""
    from apex.ops import bottleneck_bn

    torch.manual_seed(5)
    a = _chain().cuda().to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(4, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    seen = []
    conv = bottleneck_bn._conv()
    orig = conv.dgrad_bnred

    def spy(*args, **kw):
        r = orig(*args, **kw)
        seen.append(int(r[1].size(0)))
        return r

    monkeypatch.setattr(conv, "dgrad_bnred", spy, raising=False)
    monkeypatch.setattr(bottleneck_bn, "_DS_RED", True)
    ya, ga, pa, _ = _run_chain(a, x, gy, True)
    with_ds = list(seen)
    seen.clear()
    monkeypatch.setattr(bottleneck_bn, "_DS_RED", False)
    yb, gb, pb, _ = _run_chain(b, x, gy, True)
    assert sorted(with_ds) == [2, 4] and sorted(seen) == [2, 2], (with_ds, seen)
    assert torch.equal(ya, yb)
    assert _rel(ga, gb) < 1e-2, _rel(ga, gb)
    for n in pa:
        assert _rel(pa[n], pb[n]) < 1e-2, (n, _rel(pa[n], pb[n]))


@pytest.mark.gpu
def test_gpu_chain_bn1_dx_prologue_with_downsample_reduction(monkeypatch):
    """The opt-in bn1-dx prologue of conv1's dgrad (``_BN1_DX_PRO``, kProBnBwdMask) on the block
    above a downsampling block also carries that block's downsample-BN reduction (the second BN
    of the epilogue, a compile-time kernel variant since round 6): the chain runs and agrees with
    the default path to rounding."""
    from apex.ops import bottleneck_bn

    torch.manual_seed(9)
    a = _chain().cuda().to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    x = torch.randn(4, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    monkeypatch.setattr(bottleneck_bn, "_DS_RED", True)
    monkeypatch.setattr(bottleneck_bn, "_BN1_DX_PRO", True)
    ya, ga, pa, _ = _run_chain(a, x, gy, True)
    monkeypatch.setattr(bottleneck_bn, "_BN1_DX_PRO", False)
    yb, gb, pb, _ = _run_chain(b, x, gy, True)
    assert torch.equal(ya, yb)
    assert _rel(ga, gb) < 1e-2, _rel(ga, gb)
    for n in pa:
        assert _rel(pa[n], pb[n]) < 1e-2, (n, _rel(pa[n], pb[n]))
