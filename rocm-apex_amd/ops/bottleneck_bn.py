"""Training-mode ResNet bottleneck block as ONE autograd node with the batch norms fused into the
convolutions (``models.resnet.Bottleneck`` with ``fused_bn=True`` runs this on the GPU path).

Per block (M = N*H*W pixels, width w, output 4w) the forward is

    y1 = X . W1^T                + BN1 statistics in the conv epilogue   (csrc/conv/conv1x1_bn.hip)
    z1 = relu(bn1(y1))                                                   (one apply pass; at the
                                   stride-1 64 -> 64 and <= 64-pixel 3x3s it is the 3x3 conv's
                                   staged-input prologue instead, recomputed by its wgrad)
    y2 = conv3x3(z1, W2)                                                 (native implicit GEMM / MIOpen)
    BN2 statistics                                                        (one read of y2)
    y3 = relu(bn2(y2)) . W3^T    + BN3 statistics: bn2's apply+ReLU is the conv's operand
                                   prologue, so z2 is never written
    out = relu(bn3(y3) + shortcut)  (+ the ReLU bit mask)                 (one apply pass)

with shortcut = X (identity) or bn_ds(X . Wds^T) fused into the output pass (downsampling
block).  That removes two full statistics re-reads (y1: w, y3: 4w channels) and the bn2
apply pass (read + write of w channels) per block against the module-per-op path.

Backward: the bn3 reduction (bit mask, masked gradient = the identity branch's gradient),
conv3's data gradient on the native transposed-weight kernel, conv3's weight gradient on the
split-M kernel with bn2's apply+ReLU recomputed on its operand load (z2 is neither stored nor
re-materialized), bn2 / conv2 / bn1 as before, and conv1's data gradient with the shortcut's
gradient summed in (hipBLASLt ``addmm`` beta = 1), so the block hands ONE gradient tensor to
the block below — no fork.

Reference capability: apex/contrib/bottleneck (``bottleneck.cpp:1104-1534`` — the fused
scale-bias-ReLU-conv graphs with BN statistics) and groupbn's NHWC BN; the composition here is
gfx950-specific: the 1x1 convs of stages 1-2 are HBM-bound (26 GFLOP vs 0.25-0.5 GB each), so
every fused pass saved is time saved.

SyncBatchNorm (``bn_group > 1``, e.g. ``bench.py --sync-bn``): every BN of the node reduces its
statistics and backward sums over its group — one exchange per BN and direction, xGMI peer
memory or RCCL (``finalize_part`` / ``stats_pass`` / ``bwd_*``), so the fusions stay on.

``APEX_AMD_FUSED_BLOCK=0`` disables the block node (the per-module fused path runs instead).
"""
import functools
import os

import torch
import torch.nn.functional as F

from .. import _native
from . import conv as convops

_ENABLED = os.environ.get("APEX_AMD_FUSED_BLOCK", "1") != "0"
# take every native 1x1 route the kernels support, whatever the size.  The per-op routes below
# were chosen op by op in round 3 (hipBLASLt ahead on the plain stage-3/4 GEMMs); with the fused
# kernels of round 4-5 the whole-step A/B favours native everywhere: the statistics epilogue, the
# deferred output and the masked-dgrad reduction remove more standalone BN passes than the GEMM
# loses (12,404-12,410 vs 12,339-12,350 img/s same box, profiles/r05/ab_force_native_r05j.txt).
# APEX_AMD_FUSED_BLOCK_FORCE_NATIVE=0 restores the per-op routes.
FORCE_NATIVE = os.environ.get("APEX_AMD_FUSED_BLOCK_FORCE_NATIVE", "1") == "1"
_NATIVE_K = (64, 128, 256, 512)
# the deep reductions of stages 3-4 (k 1024 / 2048) on the K-streamed fused kernel
# (csrc/conv/conv1x1_ks.hip: weights through an LDS-DMA ring): conv1's / the downsample's forward
# with the statistics epilogue and conv3's data gradient with bn2's backward reduction in the
# epilogue, instead of hipBLASLt + a statistics / reduction pass.  OPT-IN (APEX_AMD_C1KS=1): the
# kernel is latency-bound at 8 waves x two 64-deep chunks of operands in flight (the 256-column
# accumulators leave no registers for a deeper ring), so the fused forms run at or behind
# hipBLASLt + the pass: stage-3 conv1 48.8 vs 36.6 + 10.6 us, conv3 dgrad + bn2 sums 57 vs
# 37 + 14.5 us (profiles/r06/resnet50_step_timeline_r06h.md), whole step -0.4 %
# (profiles/r06/ab_c1ks_r06g.txt).  The two-operand prologues (deferred output, bn3 dx:
# APEX_AMD_C1KS_PRO=1) re-read both operands per 128-column block: 128 / 109 us vs 111 / 105 us
# for the passes + hipBLASLt (profiles/r06/resnet50_step_timeline_r06f.md), -2.8 %.
_KS = os.environ.get("APEX_AMD_C1KS", "0") == "1"
_KS_PRO = os.environ.get("APEX_AMD_C1KS_PRO", "0") == "1"


def _k_native(k):
    return k in _NATIVE_K or (_KS and k % 64 == 0 and 1024 <= k <= 2048)


def _ks_only(k):
    """A deep reduction only the K-streamed kernel takes."""
    return k not in _NATIVE_K and _k_native(k)
# conv3's fused data + weight gradient (csrc/conv/conv3_bwd.hip); 0 = the two-kernel path (A/B)
_C3B = os.environ.get("APEX_AMD_CONV3_BWD", "1") != "0"
# block output pass deferred into the next block's conv1 (BlockLink.defer); 0 = A/B off
_DEFER = os.environ.get("APEX_AMD_DEFER_OUTPUT", "1") != "0"
# library 1x1 GEMMs (stage-3/4 shapes) through the hipBLASLt wrapper's timed plans
# (csrc/bindings/lt_epilogue.cpp lt_run: screened top candidates timed once per shape) instead of
# torch.matmul's single heuristic answer (+0.3 % img/s in a same-box A/B: profiles/r05/ab_rn_lt_r05f.txt)
_LT_1X1 = os.environ.get("APEX_AMD_RN_LT", "1") == "1"
# the strided 1x1 downsample as a 1x1 over the stride-2 subsample of its input (one strided copy):
# native GEMMs with the BN statistics epilogue / split-M weight gradient instead of the library's
# strided convolution, and its data gradient added at the even pixels inside conv1's dgrad
# epilogue (conv1x1_bn.hip rs_*) instead of a zero-filled dense tensor
_DS_SUB = os.environ.get("APEX_AMD_DS_SUBSAMPLE", "1") != "0"


def _lib_mm(a, b, trans_b):
    """a . op(b) for the library 1x1 routes."""
    if _LT_1X1 and a.is_cuda and a.dtype in (torch.float16, torch.bfloat16) and a.dtype == b.dtype:
        lt = _native.submodule("lt_gemm")
        if lt is not None:
            r = lt.mm(a, b, False, trans_b)
            if r:
                return r[0]
    return torch.matmul(a, b.t() if trans_b else b)


def _conv():
    return _native.require("conv").conv


# opt-in: the folded kernels are slower than the apply pass they replace on this tree — 56x56x64:
# forward 103.7 vs 111.4 us but weight gradient 137.3 vs 87.9 us, apply pass 31.5 us; 7x7x512:
# +26 / +39 us vs 8 us (tools/bn1_fold_bench.py, profiles/r05/bn1_fold_r05o.jsonl; the halo
# wgrad's in-LDS rewrite does not hide under its MFMAs yet); whole step 0 / -0.6 %
_BN1_FOLD = os.environ.get("APEX_AMD_BN1_FOLD", "0") == "1"
# bn1's dx as conv1's dgrad operand prologue with the ReLU mask recomputed from y1 (see backward)
# opt-in: same-box A/B 12,414-12,423 vs 12,508-12,532 img/s without it (profiles/r05/ab_bn1_dx_pro_r05z.txt):
# the two-operand prologue slows conv1's dgrad by more than the [M, width] pass it saves
_BN1_DX_PRO = os.environ.get("APEX_AMD_BN1_DX_PRO", "0") == "1"
# the downsample BN's dx as the downsample dgrad's operand prologue (stages 1-2, where that dgrad
# is native); 0 = reduction + dx pass + plain dgrad (A/B)
_DS_DX_PRO = os.environ.get("APEX_AMD_DS_DX_PRO", "1") != "0"
# bn1's backward reduction in the stride-1 3x3 data gradient's epilogue (conv_igemm.hip epi_chunk,
# ReLU mask recomputed from y1) instead of a reduction pass over dz1.  Opt-in: the y1 read lands in
# the per-tile epilogue of the non-persistent tap kernel, where it is exposed, and costs what the
# pass saves (same-box A/B 12,151-12,185 vs 12,160-12,205 img/s without it,
# profiles/r06/ab_bn1_red_r06k.txt)
_BN1_RED = os.environ.get("APEX_AMD_BN1_RED", "0") == "1"
# the downsample BN's backward reduction accumulated by the block above's dgrad_bnred epilogue
# (BlockLink.yd: one more operand read there instead of a reduction pass over dm and yd)
_DS_RED = os.environ.get("APEX_AMD_DS_RED", "1") != "0"


@functools.lru_cache(maxsize=None)
def _bn1_fold(cin, cout, h, w):
    """bn1's apply + ReLU folded into the stride-1 3x3 conv: its forward must run on a halo-staged
    kernel with the prologue (the 64 -> 64 spatial tile, or the halo tile where it is the default
    route: <= 64-pixel images) and its weight gradient on the halo-tile kernel (xcoef)."""
    if not _BN1_FOLD:
        return False
    fwd, dg, wg = convops.tap_route(cin, cout, 3, 1, h, w)
    if not (fwd and dg and wg and convops._halo_wgrad(cin, cout, h, w)):
        return False
    ext = _native.submodule("conv")
    if ext is None:
        return False
    sp = cin == 64 and cout == 64 and os.environ.get("APEX_AMD_CONV_SP", "1") != "0"
    hfp = (hasattr(ext, "hfp_supported") and h * w <= 64 and os.environ.get("APEX_AMD_CONV_HFP", "0")[:1] in ("1", "a")
           and bool(ext.hfp_supported(1, h, w, cin, cout)))
    return sp or hfp


class _Census:
    """APEX_AMD_BN_CENSUS=1 (diagnostics): count the node's batch-norm pass calls by (function,
    tensor shapes) and print the table at exit — maps the standalone bnh::* kernels of a trace to
    the BN they serve."""

    def __init__(self, mod):
        import atexit
        import collections

        self._mod, self._n = mod, collections.Counter()
        atexit.register(self._dump)

    def __getattr__(self, name):
        fn = getattr(self._mod, name)

        def wrap(*a, **k):
            shapes = tuple(tuple(t.shape) for t in a if isinstance(t, torch.Tensor) and t.dim() == 2)
            self._n[(name, shapes)] += 1
            return fn(*a, **k)

        return wrap

    def _dump(self):
        for (name, shapes), n in sorted(self._n.items(), key=lambda kv: -kv[1]):
            print(f"[bn census] {n:5d} {name} {shapes}", flush=True)


_CENSUS = [None]


def _bn():
    mod = _native.require("bn_nhwc").bn_nhwc
    if os.environ.get("APEX_AMD_BN_CENSUS") == "1":
        if _CENSUS[0] is None:
            _CENSUS[0] = _Census(mod)
        return _CENSUS[0]
    return mod


def _m2(t):
    """[M, C] zero-copy view of a channels_last [N, C, H, W] tensor."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.size(1))


def _nchw(t2, n, h, w):
    return t2.view(n, h, w, t2.size(1)).permute(0, 3, 1, 2)


class BlockLink:
    """Hand-off between two consecutive block nodes (block i's output feeds only block i+1).

    Forward: block i stores its output batch norm's input y3, ReLU bit mask and batch
    statistics here.  Backward: block i+1's conv1 data gradient masks its result with those bits
    and accumulates bn3_i's backward reduction in the same kernel (``dgrad_bnred``), returning
    the masked gradient and leaving the partial sums in ``part``; block i then finalizes them
    instead of re-reading its output gradient — one full read + write of the block output saved
    per block boundary.

    Forward, when the block above runs its conv1 on the native kernel (``defer``): block i does
    not run its output pass; it leaves (y3, shortcut, folded coefficients, an empty output
    tensor) in ``pend`` and block i+1's conv1 computes relu(bn3(y3) + shortcut) on its operand
    load, writing the output and its ReLU bits as by-products (``bn1x1_addrelu``) — one full read
    of the block output saved per boundary.  ``materialize`` runs the plain output pass instead
    for a consumer that does not take it."""

    __slots__ = ("y3", "bits", "mean", "invstd", "part", "defer", "pend", "yd", "meand")

    def __init__(self, defer=False):
        self.y3 = self.bits = self.mean = self.invstd = self.part = self.pend = None
        # downsampling block below: its downsample BN's input and batch mean — the same masked
        # gradient feeds that BN, so block i+1's dgrad_bnred accumulates its reduction too
        # (``part`` is then [4, G, C]: bn3's [2, G, C] slab, then the downsample BN's)
        self.yd = self.meand = None
        self.defer = defer

    def materialize(self):
        if self.pend is None:
            return
        y3, res, _, out2, c3, cd = self.pend
        self.pend = None
        o, self.bits = (_bn().apply(y3, res, c3, True, True) if cd is None
                        else _bn().apply(y3, res, c3, True, True, cd))
        out2.copy_(o)


class _BN:
    """Per-BN constants of one forward: fp32 affine params, running buffers, momentum / eps, and
    the process group its statistics are reduced over (None: this rank's batch only)."""

    __slots__ = ("w", "b", "rm", "rv", "mom", "eps", "group")

    def __init__(self, bn):
        self.w, self.b, self.rm, self.rv = bn.weight, bn.bias, bn.running_mean, bn.running_var
        self.mom, self.eps = float(bn.momentum), float(bn.eps)
        self.group = _Group(bn.process_group) if getattr(bn, "bn_group", 1) > 1 else None


class _Group:
    """Marks a synchronized BN: ``pg`` is the process group its statistics reduce over (None =
    the default group, as for torch SyncBatchNorm)."""

    __slots__ = ("pg",)

    def __init__(self, pg):
        self.pg = pg


# ---- batch statistics, local or synchronized over the BN's group (SyncBatchNorm, bn_group > 1) --
# Synchronized: each rank turns its partial sums into a Welford payload [mean | M2 | count], ONE
# exchange per BN gathers the group's payloads (xGMI peer memory, else an RCCL all-gather:
# contrib.groupbn._exchange_gather) and every member merges the same block in rank order, so all
# ranks hold bit-identical statistics (reference: optimized_sync_batchnorm_kernel.py:39 all_gather
# of [mean, var, count]).  Backward: [sum_dy | sum_dy_xmu] of every BN summed over the group
# (:104 all_reduce) before the dx coefficients; weight / bias gradients stay local (DDP averages).
def _exchange_gather(payload, group):
    from ..contrib.groupbn.batch_norm import _exchange_gather as ex

    return ex(payload, group)


def _exchange_sum(payload, group):
    from ..contrib.groupbn.batch_norm import _exchange_sum as ex

    return ex(payload, group)


def finalize_part(part, n, bn):
    """(save_mean, save_invstd, coef [2C], inv_count or None) from [2, G, C] partials about bn.rm."""
    if bn.group is None:
        sm, si, coef = _conv().bn_finalize(part, n, bn.rm, bn.w, bn.b, bn.rm, bn.rv, bn.eps, bn.mom)
        return sm, si, coef, None
    gathered = _exchange_gather(_conv().part_payload(part, n, bn.rm), bn.group.pg)
    sm, si, coef, inv_n = _bn().stats_group_merge(gathered, bn.w, bn.b, bn.rm, bn.rv, bn.mom, bn.eps)
    return sm, si, coef, inv_n


def stats_pass(y2, bn):
    """Statistics of y2 [M, C] in a pass of their own (off the epilogue-statistics conv routes)."""
    if bn.group is None:
        sm, si, coef = _bn().stats(y2, bn.w, bn.b, bn.rm, bn.rv, bn.mom, bn.eps)
        return sm, si, coef.view(-1), None
    gathered = _exchange_gather(_bn().fwd_group_local(y2), bn.group.pg)
    sm, si, coef, inv_n = _bn().stats_group_merge(gathered, bn.w, bn.b, bn.rm, bn.rv, bn.mom, bn.eps)
    return sm, si, coef, inv_n


def bwd_from_part(part, n, sm, si, w, group, inv_n):
    """(coef_bwd [3C], grad_w, grad_b) from [2, G, C] backward-reduction partials."""
    if group is None:
        return _conv().bnbwd_finalize(part, n, sm, si, w)
    payload, gw, gb = _bn().bwd_part_local(part, si)
    return _bn().bwd_group_coef(_exchange_sum(payload, group.pg), inv_n, sm, si, w), gw, gb


def bwd_reduce(dy, x, w, sm, si, coef, relu, bits, group, inv_n):
    """(dy_masked, coef_bwd, grad_w, grad_b): the reduction half of the BN backward."""
    if group is None:
        return _bn().bwd_reduce(dy, x, w, sm, si, coef, relu, bits)
    payload, gw, gb, dym = _bn().bwd_group_local(dy, x, None, w, sm, si, coef, relu, None, bits)
    return dym, _bn().bwd_group_coef(_exchange_sum(payload, group.pg), inv_n, sm, si, w), gw, gb


def bwd_full(dy, x, w, sm, si, coef, relu, group, inv_n):
    """(dx, grad_w, grad_b): reduction + dx pass."""
    if group is None:
        dx, _, gw, gb = _bn().bwd(dy, x, None, w, sm, si, coef, relu, False)
        return dx, gw, gb
    payload, gw, gb, dym = _bn().bwd_group_local(dy, x, None, w, sm, si, coef, relu)
    return _bn().bwd_group_finish(dym, x, _exchange_sum(payload, group.pg), inv_n, w, sm, si, coef), gw, gb


# ---- 1x1 stride-1 convolution pieces ---------------------------------------------------------
# Engine per op from the per-shape A/B at ResNet-50 bs 256 (profiles/bn1x1_kernels_r03a.jsonl,
# tools/bn1x1_bench.py): the native kernels run the HBM-bound stage-1/2 shapes at 4.6-6.4 TB/s
# (1.25-1.8x MIOpen / hipBLASLt); at K >= 512 with >= 256 output columns (the weight image no
# longer holds a 256-column tile) and at stage-3/4 sizes hipBLASLt is faster, so those run there
# with the separate statistics / apply passes.
def _fwd_native(m, k, n):
    if FORCE_NATIVE:
        return _k_native(k) and n % 64 == 0
    return k in _NATIVE_K and n % 64 == 0 and n <= 512 and not (k == 512 and n >= 256)


def _dgrad_native(m, kout, cin):
    if FORCE_NATIVE:
        return _k_native(kout) and cin % 64 == 0
    return kout in _NATIVE_K and cin % 64 == 0 and cin <= 256 and m >= 100000


def _red_native(m, kout, cin):
    # the masked dgrad + reduction replaces a 4-tensor-pass reduction of the block output, which
    # outweighs hipBLASLt's lead on the plain dgrad up to 512 output channels (stages 1-2)
    if FORCE_NATIVE:
        return kout in _NATIVE_K and cin % 64 == 0
    return kout in _NATIVE_K and cin % 64 == 0 and cin <= 512 and m >= 100000


def conv1x1_bn_fwd(a2, w2d, pcoef, bn):
    """y = pro(a) . W^T and the consuming BN's (save_mean, save_invstd, coef, inv_count).  pro =
    relu(a * pcoef[:K] + pcoef[K:]) when ``pcoef`` is given (the producing BN's apply + ReLU)."""
    m, k = a2.shape
    n = w2d.size(0)
    if _fwd_native(m, k, n):
        y2, part, _ = _conv().bn1x1(a2, w2d, False, pcoef, bn.rm, True)
        return (y2,) + finalize_part(part, float(m), bn)
    if pcoef is not None:
        a2 = _bn().apply(a2, None, pcoef, True)[0]
    y2 = _lib_mm(a2, w2d, True)
    return (y2,) + stats_pass(y2, bn)


def conv1x1_dgrad(g2, w2d, add2=None, add_inplace=False, sub_hw=None):
    """dX = g . W (+ add2): W [Cout, Cin], g [M, Cout].  ``add_inplace``: add2 is a temporary
    the caller no longer needs, so the library GEMM accumulates into it (beta = 1) instead of
    first copying it to a fresh output (a full D2D copy per call).  ``sub_hw = (h, w)``: add2 is
    the gradient of the stride-2 subsample of the [N, h, w] output, added at even (y, x) only."""
    m, kout = g2.shape
    # (a residual / subsampled residual is an option of the resident-weight kernel only)
    if _dgrad_native(m, kout, w2d.size(1)) and (kout in _NATIVE_K or (add2 is None and sub_hw is None)):
        h, w = sub_hw if sub_hw is not None else (0, 0)
        return _conv().bn1x1(g2, w2d, True, None, None, False, add2, res_h=h, res_w=w)[0]
    if sub_hw is not None:
        h, w = sub_hw
        dx = _lib_mm(g2, w2d, False)
        c = dx.size(1)
        dx.view(-1, h, w, c)[:, ::2, ::2].add_(add2.view(-1, (h + 1) // 2, (w + 1) // 2, c))
        return dx
    if add2 is not None:
        return add2.addmm_(g2, w2d) if add_inplace else torch.addmm(add2, g2, w2d)
    return _lib_mm(g2, w2d, False)


def conv1x1_wgrad(g2, x2, xcoef, w):
    """dW [Cout, Cin, 1, 1] = g^T . pro(x), pro = the producing BN's apply + ReLU when ``xcoef``."""
    # the split-M kernel with cost-based tiles runs 4.4-5.1 TB/s at the 56x56 shapes and leads
    # MIOpen's wgrad at every ResNet-50 1x1 shape (1.2-1.8x, profiles/bn1x1_wgrad_r03b.jsonl)
    return _conv().wgrad1x1(g2, x2, xcoef, w.dtype).view_as(w)


# ---- 3x3 / strided convolutions (ops/conv.py routes) -----------------------------------------
def _conv_fwd(x, w, stride, pad):
    fwd, _, _ = convops.tap_route(x.size(1), w.size(0), w.size(2), stride, x.size(2))
    return convops.conv_tap_forward(x, w, stride, pad) if fwd else F.conv2d(x, w, None, stride, pad)


def _conv_bwd(gy, x, w, stride, pad, need_x=True, pre=None):
    _, dg, wg = convops.tap_route(x.size(1), w.size(0), w.size(2), stride, x.size(2), x.size(3))
    dx = dw = None
    if need_x and dg:
        dx = convops.conv_tap_dgrad(gy, w, x.shape, stride, pad, pre=pre)
    if wg:
        dw = convops.conv_tap_wgrad(gy, x, w.shape, stride, pad, w.dtype)
    if (need_x and not dg) or not wg:
        dx_m, dw_m, _ = torch.ops.aten.convolution_backward(gy, x, w, None, [stride, stride], [pad, pad], [1, 1],
                                                            False, [0, 0], 1, [need_x and not dg, not wg, False])
        dx = dx if dx is not None else dx_m
        dw = dw if dw is not None else dw_m
    return dx, dw


class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, w2, w3, wds, g1, b1, g2, b2, g3, b3, gds, bds, cfg):
        bn1, bn2, bn3, bnd, stride, link_in, link_out = cfg
        n, cin, h, wd = x.shape
        width = w1.size(0)
        cout = w3.size(0)
        x2 = _m2(x)
        # conv1 (+ bn1 statistics) -> bn1 apply + ReLU; with a deferred block below, conv1 computes
        # that block's output (BN + shortcut + ReLU) on its operand load and writes it into x
        if link_in is not None and link_in.pend is not None:
            y3p, resp, pc3, outp, _, _pcd = link_in.pend
            link_in.pend = None
            DEFERRED_TAKEN[0] += 1
            y1, part1, _, link_in.bits = _conv().bn1x1_addrelu(y3p, resp, pc3, w1.view(width, cin), bn1.rm, out=outp,
                                                               split=True, res_coef=_pcd)
            sm1, si1, c1, in1 = finalize_part(part1, float(x2.size(0)), bn1)
        else:
            y1, sm1, si1, c1, in1 = conv1x1_bn_fwd(x2, w1.view(width, cin), None, bn1)
        pro1 = stride == 1 and _bn1_fold(width, w2.size(0), h, wd)
        # bn1's apply + ReLU on the 3x3 conv's staged input (and recomputed by its weight
        # gradient) instead of a pass writing z1, where both halo-staged kernels take the shape
        z1 = None if pro1 else _bn().apply(y1, None, c1, True)[0]
        # conv2 (3x3, stride) -> bn2 statistics (in the native conv's epilogue where it runs)
        z1v = _nchw(y1 if pro1 else z1, n, h, wd)
        if pro1:
            y2, part2 = convops.conv_tap_forward(z1v, w2, 1, 1, stats_shift=bn2.rm, pcoef=c1)
            oh, ow = y2.shape[2], y2.shape[3]
            y2m = _m2(y2)
            sm2, si2, c2, in2 = finalize_part(part2, float(y2m.size(0)), bn2)
        elif convops.tap_route(z1v.size(1), w2.size(0), 3, stride, h)[0]:
            y2, part2 = convops.conv_tap_forward(z1v, w2, stride, 1, stats_shift=bn2.rm)
            oh, ow = y2.shape[2], y2.shape[3]
            y2m = _m2(y2)
            sm2, si2, c2, in2 = finalize_part(part2, float(y2m.size(0)), bn2)
        else:
            y2 = F.conv2d(z1v, w2, None, stride, 1)
            oh, ow = y2.shape[2], y2.shape[3]
            y2m = _m2(y2)
            sm2, si2, c2, in2 = stats_pass(y2m, bn2)
        # conv3 with bn2's apply + ReLU on its operand load (+ bn3 statistics)
        y3, sm3, si3, c3, in3 = conv1x1_bn_fwd(y2m, w3.view(cout, width), c2, bn3)
        yd = smd = sid = cd = ind = xs2 = None
        if wds is not None:
            if stride == 1:
                yd, smd, sid, cd, ind = conv1x1_bn_fwd(x2, wds.view(cout, cin), None, bnd)
            elif _DS_SUB and stride == 2 and wds.size(2) == 1:
                xs2 = _conv().subsample2x(x2, n, h, wd)
                yd, smd, sid, cd, ind = conv1x1_bn_fwd(xs2, wds.view(cout, cin), None, bnd)
            else:
                yd = _m2(_conv_fwd(x, wds, stride, 0))
                smd, sid, cd, ind = stats_pass(yd, bnd)
        if link_out is not None and link_out.defer:
            # the block above computes this output in its conv1 (BlockLink docstring)
            res = x2 if wds is None else yd
            # the consumer's prologue takes bn3's [scale | shift] and the downsample BN's (None: the
            # identity shortcut, scale 1 / shift 0) and assembles [a scale | res scale | a shift |
            # res shift] on its LDS load: the apply passes' arithmetic exactly, no concatenation
            out2, bits = torch.empty_like(y3), None
            link_out.pend = (y3, res, c3, out2, c3, cd)
        elif wds is None:
            out2, bits = _bn().apply(y3, x2, c3, True, True)
        else:
            out2, bits = _bn().apply(y3, yd, c3, True, True, cd)
        ctx.save_for_backward(x, w1, w2, w3, wds, g1, g2, g3, gds, y1, z1, y2m, y3, yd, bits,
                              sm1, si1, c1, sm2, si2, c2, sm3, si3, c3, smd, sid, cd, in1, in2, in3, ind, xs2)
        ctx.geo = (n, h, wd, oh, ow, stride)
        ctx.links = (link_in, link_out)
        # the 3x3 data gradient's weight images, built on a side stream under this forward
        ctx.pre2 = (convops.tap_images_async(w2, (n, width, h, wd), stride, 1)
                    if pro1 or convops.tap_route(width, w2.size(0), 3, stride, h, wd)[1] else None)
        ctx.groups = (bn1.group, bn2.group, bn3.group, bnd.group if bnd is not None else None)
        if link_out is not None:
            link_out.y3, link_out.bits, link_out.mean, link_out.invstd = y3, bits, sm3, si3
            if wds is not None and _DS_RED:
                link_out.yd, link_out.meand = yd, smd
        return _nchw(out2, n, oh, ow)

    @staticmethod
    def backward(ctx, gout):
        (x, w1, w2, w3, wds, g1, g2, g3, gds, y1, z1, y2m, y3, yd, bits,
         sm1, si1, c1, sm2, si2, c2, sm3, si3, c3, smd, sid, cd, in1, in2, in3, ind, xs2) = ctx.saved_tensors
        n, h, wd, oh, ow, stride = ctx.geo
        gr1, gr2, gr3, grd = ctx.groups
        bn = _bn()
        width, cin, cout = w1.size(0), w1.size(1), w3.size(0)
        gout = gout.contiguous(memory_format=torch.channels_last)
        go2 = _m2(gout)
        x2 = _m2(x)
        link_in, link_out = ctx.links
        # bn3 (+ shortcut): masked gradient dm (= the identity branch's gradient) + coefficients
        # (the block above already masked the gradient and reduced it when linked); bn3's dx
        # pass runs as conv3's dgrad operand prologue (dx3 written as a by-product for the
        # weight gradient) where that kernel takes the shape
        ds_part = None
        if link_out is not None and link_out.part is not None:
            dm = go2
            part = link_out.part
            if part.size(0) == 4:  # the downsample BN's reduction came along (BlockLink.yd)
                part, ds_part = part[0:2], part[2:4]
            cb3, gg3, gb3 = bwd_from_part(part, float(go2.size(0)), sm3, si3, g3, gr3, in3)
            link_out.part = None
        else:
            if bits is None:  # deferred output: its ReLU bits came from the block above's conv1
                bits = link_out.bits
            dm, cb3, gg3, gb3 = bwd_reduce(go2, y3, g3, sm3, si3, c3, True, bits, gr3, in3)
        w3m = w3.view(cout, width)
        dw3 = None
        if _C3B and _conv().supports_conv3_bwd(cout, width):
            # conv3's data AND weight gradients in one pass (csrc/conv/conv3_bwd.hip): bn3's dx
            # computed on the operand load and kept in LDS, bn2's ReLU mask + backward sums in the
            # dgrad epilogue, bn2's apply+ReLU on the weight gradient's operand
            dz2, part2, dw3 = _conv().conv3_bwd(dm, y3, y2m, w3m, cb3.view(-1), c2, sm2)
            dw3 = dw3.view_as(w3)
            cb2, gg2, gb2 = bwd_from_part(part2, float(dm.size(0)), sm2, si2, g2, gr2, in2)
            dy2 = bn.bwd_apply(dz2, y2m, c2, cb2)
        elif _dgrad_native(dm.size(0), cout, width) and _ks_only(cout) and not _KS_PRO:
            # stages 3-4 (K-streamed kernel): bn3's dx pass, then conv3's dgrad with bn2's ReLU mask
            # recomputed and its backward sums in the epilogue (no bn2 reduction pass)
            dx3 = bn.bwd_apply(dm, y3, c3, cb3)
            dz2, part2, _ = _conv().dgrad_bnred(dx3, w3m, None, None, y2m, sm2, coef=c2)
            cb2, gg2, gb2 = bwd_from_part(part2, float(dm.size(0)), sm2, si2, g2, gr2, in2)
            dy2 = bn.bwd_apply(dz2, y2m, c2, cb2)
        elif _dgrad_native(dm.size(0), cout, width) and (width == 64 or _ks_only(cout)):
            # conv3 dgrad with bn3's dx as the operand prologue (dx3 written for the wgrad) AND
            # bn2's ReLU mask + backward reduction in the epilogue: bn2's reduction pass is gone
            # (stage 1 only: at 128+ channels the longer epilogue costs more than the pass,
            # profiles/resnet50_node_r03e.md; and stages 3-4 on the K-streamed kernel, whose
            # epilogue runs under the deep reduction's MFMAs)
            dz2, part2, dx3 = _conv().dgrad_bnred(dm, w3m, None, None, y2m, sm2, coef=c2, py=y3,
                                                  pcoef=cb3.view(-1), want_aout=True)
            cb2, gg2, gb2 = bwd_from_part(part2, float(dm.size(0)), sm2, si2, g2, gr2, in2)
            dy2 = bn.bwd_apply(dz2, y2m, c2, cb2)
        elif _dgrad_native(dm.size(0), cout, width):
            dz2, _, dx3 = _conv().bn1x1(dm, w3m, True, cb3.view(-1), None, False, None, y3, True)
            dy2, gg2, gb2 = bwd_full(dz2, y2m, g2, sm2, si2, c2, True, gr2, in2)
        else:
            dx3 = bn.bwd_apply(dm, y3, c3, cb3)
            dz2 = conv1x1_dgrad(dx3, w3m)
            dy2, gg2, gb2 = bwd_full(dz2, y2m, g2, sm2, si2, c2, True, gr2, in2)
        # conv3 weight gradient with bn2's apply + ReLU recomputed on the operand load
        if dw3 is None:
            dw3 = conv1x1_wgrad(dx3, y2m, c2, w3)
        # conv2
        # stride-1 3x3 dgrad on the tap kernels (width > 64: stage 1's 64 -> 64 runs the spatial
        # kernel, which has no reduction epilogue), a local BN (the group exchange takes the pass)
        red1 = (_BN1_RED and z1 is not None and stride == 1 and width > 64 and gr1 is None
                and convops.tap_route(width, w2.size(0), 3, 1, h, wd)[1])
        if z1 is None:  # bn1 folded into the 3x3 conv: its weight gradient recomputes z1 from y1
            gy2 = _nchw(dy2, n, oh, ow)
            dz1 = convops.conv_tap_dgrad(gy2, w2, (n, width, h, wd), 1, 1, pre=ctx.pre2)
            dw2 = convops.conv_tap_wgrad(gy2, _nchw(y1, n, h, wd), w2.shape, 1, 1, w2.dtype, xcoef=c1)
        elif red1:
            # bn1's backward reduction in the 3x3 dgrad's epilogue (ReLU mask recomputed from y1):
            # dz1 comes out masked with its [2, tiles, width] sums, no reduction pass over it
            gy2 = _nchw(dy2, n, oh, ow)
            dz1, part1 = convops.conv_tap_dgrad(gy2, w2, (n, width, h, wd), 1, 1, red=(_nchw(y1, n, h, wd), c1, sm1),
                                                pre=ctx.pre2)
            dw2 = _conv_bwd(gy2, _nchw(z1, n, h, wd), w2, stride, 1, need_x=False)[1]
        else:
            dz1, dw2 = _conv_bwd(_nchw(dy2, n, oh, ow), _nchw(z1, n, h, wd), w2, stride, 1, pre=ctx.pre2)
        dz1 = _m2(dz1.contiguous(memory_format=torch.channels_last))
        # bn1: the reduction pass only, its dx as conv1's dgrad operand prologue with the ReLU mask
        # recomputed from y1 (kProBnBwdMask: the reduction writes nothing, the prologue writes dy1
        # for the weight gradient — one [M, width] pass fewer than reduction + dx + dgrad reading
        # dy1); bwd_full where conv1's dgrad is not native or the BN is synchronized, and at width
        # 512 (stage 4: the 5 coefficient rows next to the 128 x 512 weight image exceed the LDS)
        bn1_pro = (_BN1_DX_PRO and not red1 and gr1 is None and width <= 256
                   and _dgrad_native(dz1.size(0), width, cin))
        if red1:  # dz1 is already masked: bn1's coefficients from the epilogue partials, then its dx
            cb1, gg1, gb1 = bwd_from_part(part1, float(dz1.size(0)), sm1, si1, g1, gr1, in1)
            dy1 = bn.bwd_apply(dz1, y1, c1, cb1)
        elif bn1_pro:
            pc1, gg1, gb1 = bn.bwd_coef(dz1, y1, g1, sm1, si1, c1)
            pc1 = pc1.view(-1)
        else:
            dy1, gg1, gb1 = bwd_full(dz1, y1, g1, sm1, si1, c1, True, gr1, in1)
        # shortcut gradient, then conv1's data gradient summed onto it
        dwd = ggd = gbd = None
        sub_hw = None  # (h, w): ``short`` is the subsampled downsample gradient (see _DS_SUB)
        if wds is None:
            # dm is this node's own temporary unless the block above handed it in (then it is
            # autograd's incoming gradient, which must not be written)
            short = dm
            short_tmp = dm is not go2
        else:
            short_tmp = True
            # the downsample BN's dx as the downsample dgrad's operand prologue (kProBnBwd: the
            # reduction pass writes nothing, the prologue writes dyd for the weight gradient) —
            # one [M, cout] pass and a launch fewer than reduction + dx pass + dgrad reading dyd
            ds_pro = (_DS_DX_PRO and (grd is None or ds_part is not None) and (stride == 1 or xs2 is not None)
                      and _dgrad_native(dm.size(0), cout, cin) and (cout in _NATIVE_K or _KS_PRO))
            if ds_part is not None:  # reduced by the block above's dgrad_bnred epilogue
                cbd, ggd, gbd = bwd_from_part(ds_part, float(dm.size(0)), smd, sid, gds, grd, ind)
            elif ds_pro:
                _, cbd, ggd, gbd = bn.bwd_reduce(dm, yd, gds, smd, sid, cd, False, None)
            if ds_pro:
                short, _, dyd = _conv().bn1x1(dm, wds.view(cout, cin), True, cbd.view(-1), None, False, None, yd, True)
            elif ds_part is not None:
                dyd = bn.bwd_apply(dm, yd, cd, cbd)
            else:
                dyd, ggd, gbd = bwd_full(dm, yd, gds, smd, sid, cd, False, grd, ind)
            if stride == 1:
                if not ds_pro:
                    short = conv1x1_dgrad(dyd, wds.view(cout, cin))
                dwd = conv1x1_wgrad(dyd, x2, None, wds)
            elif xs2 is not None:
                if not ds_pro:
                    short = conv1x1_dgrad(dyd, wds.view(cout, cin))
                dwd = conv1x1_wgrad(dyd, xs2, None, wds)
                sub_hw = (h, wd)
            else:
                dxd, dwd = _conv_bwd(_nchw(dyd, n, oh, ow), x, wds, stride, 0)
                short = _m2(dxd.contiguous(memory_format=torch.channels_last))
        rh, rw = sub_hw if sub_hw is not None else (0, 0)
        if link_in is not None and link_in.bits is not None and _red_native(dz1.size(0), width, cin):
            # mask with the block below's ReLU bits + its bn3 backward reduction, in this kernel
            ds2 = dict(x2=link_in.yd, mean2=link_in.meand) if link_in.yd is not None else {}
            if bn1_pro:
                dx, link_in.part, dy1 = _conv().dgrad_bnred(dz1, w1.view(width, cin), short, link_in.bits, link_in.y3,
                                                            link_in.mean, py=y1, pcoef=pc1, want_aout=True, res_h=rh,
                                                            res_w=rw, **ds2)
            else:
                dx, link_in.part, _ = _conv().dgrad_bnred(dy1, w1.view(width, cin), short, link_in.bits, link_in.y3,
                                                          link_in.mean, res_h=rh, res_w=rw, **ds2)
            link_in.yd = link_in.meand = None
        elif bn1_pro:
            dx, _, dy1 = _conv().bn1x1(dz1, w1.view(width, cin), True, pc1, None, False, short, y1, True, res_h=rh,
                                       res_w=rw)
        else:
            dx = conv1x1_dgrad(dy1, w1.view(width, cin), short, short_tmp, sub_hw)
        dw1 = conv1x1_wgrad(dy1, x2, None, w1)
        return (_nchw(dx, n, h, wd), dw1, dw2, dw3, dwd, gg1, gb1, gg2, gb2, gg3, gb3, ggd, gbd, None)


def _bn_ok(bn):
    # any bn_group: with bn_group > 1 (SyncBatchNorm over bn.process_group) the statistics and
    # backward sums are exchanged per BN (finalize_part / stats_pass / bwd_* above)
    return (bn.training and bn.track_running_stats and bn.weight is not None
            and bn.weight.dtype == torch.float32 and bn.momentum is not None and bn.running_mean is not None)


def block_supported(block, x):
    """True when ``block`` (a fused_bn Bottleneck) can run as one fused node on ``x``."""
    if not (_ENABLED and torch.is_tensor(x) and x.is_cuda and x.dim() == 4 and _native.available()
            and x.dtype in (torch.bfloat16, torch.float16) and x.is_contiguous(memory_format=torch.channels_last)
            and not torch.is_autocast_enabled("cuda")):
        return False
    if _native.submodule("conv") is None or _native.submodule("bn_nhwc") is None:
        return False
    convs = [block.conv1, block.conv2, block.conv3]
    bns = [block.bn1, block.bn2, block.bn3]
    if block.downsample is not None:
        convs.append(block.downsample[0])
        bns.append(block.downsample[1])
    if not all(_bn_ok(b) for b in bns):
        return False
    if not all(c.weight.dtype == x.dtype and c.bias is None and c.groups == 1 and c.dilation == (1, 1)
               and c.weight.is_contiguous(memory_format=torch.channels_last) for c in convs):
        return False
    if block.conv2.kernel_size != (3, 3) or block.conv1.stride != (1, 1) or block.conv3.stride != (1, 1):
        return False
    chans = (block.conv1.in_channels, block.conv1.out_channels, block.conv3.out_channels)
    return all(c % 64 == 0 for c in chans)


def takes_deferred_input(block, x_shape, dtype):
    """True when ``block`` (the next fused node) will run its conv1 on the native kernel, so the
    block below may defer its output pass to it (``BlockLink.defer``)."""
    if not (_DEFER and _ENABLED and getattr(block, "fused_bn", False) and block.training):
        return False
    if dtype not in (torch.bfloat16, torch.float16) or block.conv1.weight.dtype != dtype:
        return False
    n, c, h, w = x_shape
    width = block.conv1.out_channels
    # (the deep stage-3 / 4 reductions take the deferred output only with the K-streamed kernel's
    # two-operand prologue, _KS_PRO)
    return (block.conv1.in_channels == c and _fwd_native(n * h * w, c, width) and (c in _NATIVE_K or _KS_PRO)
            and _bn_ok(block.bn1))


# block outputs computed by the next block's conv1 (BlockLink.defer) since import
DEFERRED_TAKEN = [0]

# forward calls of the node since import (bench.py reports nodes per step)
NODE_CALLS = [0]


def bottleneck_forward(block, x, link_in=None, link_out=None):
    """Run ``block`` as one node.  ``link_in``: the BlockLink the block below filled (its output
    is ``x`` and feeds nothing else); ``link_out``: a fresh BlockLink for the block above."""
    NODE_CALLS[0] += 1
    ds = block.downsample
    stride = block.conv2.stride[0]
    if ds is not None and ds[0].stride[0] != stride:
        raise ValueError("fused bottleneck: downsample stride must match conv2's")
    cfg = (_BN(block.bn1), _BN(block.bn2), _BN(block.bn3), _BN(ds[1]) if ds is not None else None, stride,
           link_in, link_out)
    return _BottleneckFn.apply(
        x, block.conv1.weight, block.conv2.weight, block.conv3.weight, ds[0].weight if ds is not None else None,
        block.bn1.weight, block.bn1.bias, block.bn2.weight, block.bn2.bias, block.bn3.weight, block.bn3.bias,
        ds[1].weight if ds is not None else None, ds[1].bias if ds is not None else None, cfg)
