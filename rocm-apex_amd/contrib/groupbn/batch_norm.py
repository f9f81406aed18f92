"""NHWC batch norm with fused ReLU and fused residual add + ReLU
(reference apex/contrib/groupbn/batch_norm.py:24-260 — ``BatchNorm2d_NHWC``).

GPU path: the gfx950 fused pipeline in ``csrc/groupbn/bn_nhwc.hip`` (3 passes forward, 5
backward, ReLU mask recomputed in registers, deterministic partial reductions).  The module
accepts either a logical NHWC tensor ``[N, H, W, C]`` or — with ``torch_channels_last=True`` — an
NCHW-shaped tensor in ``torch.channels_last`` memory (what convolutions produce); both are handed
to the kernels as the same zero-copy ``[M, C]`` view and the output keeps the input's layout.

``bn_group > 1`` (statistics shared by groups of adjacent ranks; the reference does this through
CUDA-IPC peer memory and compiles it out on HIP): the SAME fused kernels run in two halves around
one tiny exchange per direction (``_BnNHWCGroupFunction``):

* forward: stats pass -> local payload [mean | M2 | count] (2C+1 floats) -> exchange -> a merge
  kernel that combines the group's payloads in rank order (identical result on every member) and
  writes the apply constants -> the fused apply pass (+z, +ReLU, +ReLU bit mask);
* backward: reduction pass (masking, second-gradient sum) -> local [sum_dy | sum_dy_xmu] ->
  exchange -> coefficient kernel -> the fused dx pass.

The exchange is a hipIpc peer-memory push/flag-wait kernel over xGMI (``apex.parallel.peer_memory``,
one single-workgroup launch, no RCCL protocol round trip per layer) or, with ``peer_memory=False``
/ no peer support, an RCCL sub-group ``all_gather_into_tensor`` / ``all_reduce``.  Weight / bias
gradients stay LOCAL (the data-parallel reduction averages them like every other gradient), as in
the reference's SyncBatchNorm.  CPU tensors and channel counts that are not a multiple of 8 use the
generic SyncBatchNorm primitives.
"""
import os

import torch
from torch.nn.modules.batchnorm import _BatchNorm

from ... import _native
from ...ops import batchnorm as bnops


# APEX_BN_BITS=0: recompute the residual ReLU mask from x and z in backward instead (A/B switch)
_BITS = os.environ.get("APEX_BN_BITS", "1") != "0"


def _ext():
    return _native.require("bn_nhwc").bn_nhwc


def _to_2d(t, torch_channels_last):
    """[M, C] zero-copy view of an NHWC tensor (logical NHWC, or NCHW-shaped channels_last)."""
    if t is None:
        return None
    if torch_channels_last and t.dim() == 4:
        if not t.is_contiguous(memory_format=torch.channels_last):
            t = t.contiguous(memory_format=torch.channels_last)
        c = t.size(1)
        return t.permute(0, 2, 3, 1).reshape(-1, c)
    t = t.contiguous()
    return t.view(-1, t.size(-1))


def _from_2d(t2d, like, torch_channels_last):
    if torch_channels_last and like.dim() == 4:
        n, c, h, w = like.shape
        return t2d.view(n, h, w, c).permute(0, 3, 1, 2)
    return t2d.view(like.shape)


class _BnNHWCFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, training,
                torch_channels_last, fork=False):
        ctx.set_materialize_grads(False)
        x2 = _to_2d(x, torch_channels_last)
        z2 = _to_2d(z, torch_channels_last)
        ext = _ext()
        if training:
            # residual add + ReLU: the forward also writes the ReLU mask as bits and the backward
            # reads those instead of z (z is not kept alive for this layer's backward at all)
            bits = _BITS and bool(fuse_relu) and z2 is not None
            y2, save_mean, save_invstd, coef, mask = ext.fwd_train(x2, z2, weight, bias, running_mean, running_var,
                                                                   float(momentum), float(eps), bool(fuse_relu),
                                                                   bits)
            ctx.save_for_backward(x2, None if bits else z2, weight, save_mean, save_invstd, coef,
                                  mask if bits else None)
        else:
            y2 = ext.fwd_eval(x2, z2, weight, bias, running_mean, running_var, float(eps), bool(fuse_relu))
            ctx.save_for_backward(x2, z2, weight, None, None, None, None)
        ctx.fuse_relu = fuse_relu
        ctx.training = training
        ctx.has_z = z is not None
        ctx.layout = (torch_channels_last, x.shape, x.dim())
        y = _from_2d(y2, x, torch_channels_last)
        if fork:
            # two aliases of one output for two consumers (a residual block's main and shortcut
            # branches): autograd hands their gradients to backward separately and the reduction
            # kernel sums them in registers — no separate gradient-add pass over the activation
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, grad_y, grad_y2=None):
        x2, z2, weight, save_mean, save_invstd, coef, mask = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("BatchNorm2d_NHWC: backward through an eval-mode forward is not supported")
        if grad_y is None:
            grad_y, grad_y2 = grad_y2, None
        if grad_y is None:
            return (None,) * 12
        tcl, shape, _ = ctx.layout
        g2 = _to_2d(grad_y, tcl)
        gg2 = _to_2d(grad_y2, tcl) if grad_y2 is not None else None
        need_dz = ctx.has_z and ctx.needs_input_grad[1]
        dx2, dz2, gw, gb = _ext().bwd(g2, x2, z2, weight, save_mean, save_invstd, coef, bool(ctx.fuse_relu),
                                      bool(need_dz), gg2, mask)
        like = torch.empty(shape, device="meta")
        dx = _from_2d(dx2, like, tcl)
        dz = _from_2d(dz2, like, tcl) if need_dz else None
        gw = gw if (weight is not None and ctx.needs_input_grad[2]) else None
        gb = gb if (weight is not None and ctx.needs_input_grad[3]) else None
        return dx, dz, gw, gb, None, None, None, None, None, None, None, None


class _BnDualAddReluFunction(torch.autograd.Function):
    """y = relu(bn_x(x) + bn_z(z)) for a residual block whose shortcut is conv -> BN: statistics of
    both inputs, then ONE output pass (``fwd_train_dual``) — the shortcut's normalized tensor is
    never materialized.  Backward: the main BN's reduction writes the ReLU-masked gradient (read
    from the forward's bit mask), which is at once the shortcut BN's incoming gradient."""

    @staticmethod
    def forward(ctx, x, z, w, b, rm, rv, wz, bz, rmz, rvz, momentum, eps, momentum_z, eps_z, torch_channels_last,
                fork=False):
        ctx.set_materialize_grads(False)
        x2 = _to_2d(x, torch_channels_last)
        z2 = _to_2d(z, torch_channels_last)
        y2, sm, si, coef, smz, siz, coefz, mask = _ext().fwd_train_dual(
            x2, z2, w, b, rm, rv, float(momentum), float(eps), wz, bz, rmz, rvz, float(momentum_z), float(eps_z), True)
        ctx.save_for_backward(x2, z2, w, sm, si, coef, wz, smz, siz, coefz, mask)
        ctx.layout = (torch_channels_last, x.shape)
        y = _from_2d(y2, x, torch_channels_last)
        if fork:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, grad_y, grad_y2=None):
        x2, z2, w, sm, si, coef, wz, smz, siz, coefz, mask = ctx.saved_tensors
        if grad_y is None:
            grad_y, grad_y2 = grad_y2, None
        if grad_y is None:
            return (None,) * 16
        tcl, shape = ctx.layout
        g2 = _to_2d(grad_y, tcl)
        gg2 = _to_2d(grad_y2, tcl) if grad_y2 is not None else None
        ext = _ext()
        dx2, dym, gw, gb = ext.bwd(g2, x2, None, w, sm, si, coef, True, True, gg2, mask)
        dz2, _, gwz, gbz = ext.bwd(dym, z2, None, wz, smz, siz, coefz, False, False)
        like = torch.empty(shape, device="meta")
        return (_from_2d(dx2, like, tcl), _from_2d(dz2, like, tcl), gw, gb, None, None, gwz, gbz, None, None, None,
                None, None, None, None, None)


def bn_add_bn_relu(x, z, bn_x, bn_z, fork=False):
    """``relu(bn_x(x) + bn_z(z))`` — the output of a downsampling residual block — as one fused
    output pass when both are single-rank training-mode BatchNorm2d_NHWC on the native path;
    otherwise the two modules in sequence (bn_z first, its output as bn_x's residual input)."""
    ok = (bn_x.training and bn_z.training and bn_x.fuse_relu and not bn_z.fuse_relu and bn_x.bn_group == 1
          and bn_z.bn_group == 1 and bn_x.torch_channels_last and bn_z.torch_channels_last
          and x.dim() == 4 and z.shape == x.shape and z.dtype == x.dtype and _native.use_native(x)
          and x.size(1) % 8 == 0 and bn_x.weight is not None and bn_z.weight is not None
          and bn_x.weight.dtype == torch.float32 and bn_z.weight.dtype == torch.float32
          and bn_x.track_running_stats and bn_z.track_running_stats)
    if not ok:
        return bn_x(x, bn_z(z), fork=fork)
    return _BnDualAddReluFunction.apply(x, z, bn_x.weight, bn_x.bias, bn_x.running_mean, bn_x.running_var,
                                        bn_z.weight, bn_z.bias, bn_z.running_mean, bn_z.running_var, bn_x.momentum,
                                        bn_x.eps, bn_z.momentum, bn_z.eps, True, fork)


class _BnReluMaxPoolFunction(torch.autograd.Function):
    """maxpool(relu(bn(x))) for the ResNet stem: BN statistics, then ONE pass that normalizes,
    applies the ReLU and pools (``fwd_train_relu_maxpool``), so the full-resolution activation is
    only read once and never written.  Backward: the NHWC pool's gather backward (1-byte window
    indices) gives the gradient of the BN+ReLU output, then the fused BN backward with the ReLU
    mask recomputed from x."""

    @staticmethod
    def forward(ctx, x, w, b, rm, rv, momentum, eps, k, st, pad):
        y, idx, sm, si, coef = _ext().fwd_train_relu_maxpool(x, w, b, rm, rv, float(momentum), float(eps), list(k),
                                                             list(st), list(pad))
        ctx.save_for_backward(x, w, sm, si, coef, idx)
        ctx.pool = (k, st, pad)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, gp):
        x, w, sm, si, coef, idx = ctx.saved_tensors
        k, st, pad = ctx.pool
        gy = _native.require("maxpool_nhwc").maxpool_nhwc.backward(gp, idx, x, list(k), list(st), list(pad))
        dx2, _, gw, gb = _ext().bwd(_to_2d(gy, True), _to_2d(x, True), None, w, sm, si, coef, True, False)
        like = torch.empty(x.shape, device="meta")
        return _from_2d(dx2, like, True), gw, gb, None, None, None, None, None, None, None


def bn_relu_maxpool(x, bn, pool):
    """``pool(bn(x))`` for a ReLU-fused training-mode ``BatchNorm2d_NHWC`` followed by a max pool
    (the ResNet stem) in one fused pass on the native path; otherwise the two modules in turn."""
    def _pair(v):
        return (v, v) if isinstance(v, int) else tuple(v)

    k, st, pad = _pair(pool.kernel_size), _pair(pool.stride if pool.stride is not None else pool.kernel_size), \
        _pair(pool.padding)
    ok = (bn.training and bn.fuse_relu and bn.bn_group == 1 and bn.torch_channels_last and x.dim() == 4
          and x.is_contiguous(memory_format=torch.channels_last) and _native.use_native(x) and x.size(1) % 8 == 0
          and bn.weight is not None and bn.weight.dtype == torch.float32 and bn.track_running_stats
          and getattr(pool, "dilation", 1) in (1, (1, 1)) and not getattr(pool, "ceil_mode", False)
          and not getattr(pool, "return_indices", False) and _native.submodule("maxpool_nhwc") is not None)
    if not ok:
        return pool(bn(x))
    return _BnReluMaxPoolFunction.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                                        k, st, pad)


def _exchange_gather(payload, group):
    """[world, n] fp32: every group member's ``payload`` (peer memory, else RCCL / gloo)."""
    from ...parallel import comm_timing

    with comm_timing.span("bn_exchange", payload.device):
        return _exchange_gather_impl(payload, group)


def _exchange_gather_impl(payload, group):
    import torch.distributed as dist

    from ...parallel.peer_memory import get_peer_exchange

    peer = get_peer_exchange(group)
    if peer is not None:
        return peer.all_gather(payload)
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world, payload.numel(), dtype=payload.dtype, device=payload.device)
        dist.all_gather_into_tensor(out, payload, group=group)
        return out
    host = payload.cpu()  # gloo (rehearsal / tests): host staging
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    return torch.stack(parts, 0).to(payload.device)


def _exchange_sum(payload, group):
    """Group sums as [rows, n] rows to be added in order by the consumer kernel: the peer path
    hands back every member's row (summed in rank order in-kernel, identical on all members),
    the collective path one all-reduced row."""
    from ...parallel import comm_timing

    with comm_timing.span("bn_exchange", payload.device):
        return _exchange_sum_impl(payload, group)


def _exchange_sum_impl(payload, group):
    import torch.distributed as dist

    from ...parallel.peer_memory import get_peer_exchange

    peer = get_peer_exchange(group)
    if peer is not None:
        return peer.all_gather(payload)
    if dist.get_backend(group) == "nccl":
        out = payload.clone()
        dist.all_reduce(out, dist.ReduceOp.SUM, group=group)
        return out.view(1, -1)
    host = payload.cpu()
    dist.all_reduce(host, dist.ReduceOp.SUM, group=group)
    return host.to(payload.device).view(1, -1)


class _BnNHWCGroupFunction(torch.autograd.Function):
    """bn_group > 1: fused NHWC batch norm with the statistics reduced over ``group``."""

    @staticmethod
    def forward(ctx, x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, group,
                torch_channels_last, fork=False):
        ctx.set_materialize_grads(False)
        x2 = _to_2d(x, torch_channels_last)
        z2 = _to_2d(z, torch_channels_last)
        ext = _ext()
        gathered = _exchange_gather(ext.fwd_group_local(x2), group)
        bits = bool(fuse_relu) and z2 is not None
        y2, save_mean, save_invstd, coef, mask, inv_count = ext.fwd_group_finish(
            x2, z2, gathered, weight, bias, running_mean, running_var, float(momentum), float(eps), bool(fuse_relu),
            bits)
        ctx.save_for_backward(x2, None if bits else z2, weight, save_mean, save_invstd, coef,
                              mask if bits else None, inv_count)
        ctx.fuse_relu = fuse_relu
        ctx.has_z = z is not None
        ctx.group = group
        ctx.layout = (torch_channels_last, x.shape)
        y = _from_2d(y2, x, torch_channels_last)
        if fork:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, grad_y, grad_y2=None):
        x2, z2, weight, save_mean, save_invstd, coef, mask, inv_count = ctx.saved_tensors
        if grad_y is None:
            grad_y, grad_y2 = grad_y2, None
        if grad_y is None:
            # every member must still join the exchange: contribute zero gradient sums
            grad_y = torch.zeros_like(x2)
            g2 = grad_y
        else:
            g2 = _to_2d(grad_y, ctx.layout[0])
        gg2 = _to_2d(grad_y2, ctx.layout[0]) if grad_y2 is not None else None
        ext = _ext()
        payload, gw, gb, dym = ext.bwd_group_local(g2, x2, z2, weight, save_mean, save_invstd, coef,
                                                   bool(ctx.fuse_relu), gg2, mask)
        sums = _exchange_sum(payload, ctx.group)
        dx2 = ext.bwd_group_finish(dym, x2, sums, inv_count, weight, save_mean, save_invstd, coef)
        tcl, shape = ctx.layout
        like = torch.empty(shape, device="meta")
        dx = _from_2d(dx2, like, tcl)
        dz = None
        if ctx.has_z and ctx.needs_input_grad[1]:
            dz = _from_2d(dym, like, tcl)
        gw = gw if (weight is not None and ctx.needs_input_grad[2]) else None
        gb = gb if (weight is not None and ctx.needs_input_grad[3]) else None
        return dx, dz, gw, gb, None, None, None, None, None, None, None, None


def _reference_bn(x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, training, channels_last_dim):
    """torch / generic-kernel path (CPU, C % 8 != 0): SyncBatchNorm primitives on an [M, C] view."""
    from ...parallel.optimized_sync_batchnorm import SyncBatchnormFunction

    return SyncBatchnormFunction.apply(x, z, weight, bias, running_mean, running_var, eps, training, momentum,
                                       "local", channels_last_dim, fuse_relu)


def bn_nhwc_function(x, z, weight, bias, running_mean, running_var, momentum=0.1, eps=1e-5, fuse_relu=False,
                     training=True, torch_channels_last=True, fork=False):
    """``fork=True`` returns ``(y, y_alias)``: one output for two consumers whose gradients the
    fused backward sums itself (ResNet blocks hand the alias to the next block's shortcut)."""
    c = x.size(1) if (torch_channels_last and x.dim() == 4) else x.size(-1)
    if _native.use_native(x) and c % 8 == 0 and weight is not None and weight.dtype == torch.float32:
        return _BnNHWCFunction.apply(x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu,
                                     training, torch_channels_last, fork)
    y = _bn_generic(x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, training,
                    torch_channels_last)
    return (y, y) if fork else y


def _bn_generic(x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, training,
                torch_channels_last):
    if torch_channels_last and x.dim() == 4:
        xv = x.permute(0, 2, 3, 1)
        zv = z.permute(0, 2, 3, 1) if z is not None else None
        y = _reference_bn(xv, zv, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, training, True)
        return y.permute(0, 3, 1, 2)
    return _reference_bn(x, z, weight, bias, running_mean, running_var, momentum, eps, fuse_relu, training, True)


class BatchNorm2d_NHWC(_BatchNorm):
    """``BatchNorm2d_NHWC(num_features, fuse_relu=False, bn_group=1, torch_channels_last=False,
    max_cta_per_sm=2, cta_launch_margin=12, multi_stream=False)``; ``forward(x, z=None)``
    computes ``relu(bn(x) + z)`` when ``z`` is given (requires ``fuse_relu``).

    ``max_cta_per_sm`` / ``cta_launch_margin`` / ``multi_stream`` tune the reference's persistent
    CUDA kernels and are accepted for API compatibility (the gfx950 kernels size their grids
    from the CU count)."""

    def __init__(self, num_features, fuse_relu=False, bn_group=1, torch_channels_last=False, max_cta_per_sm=2,
                 cta_launch_margin=12, multi_stream=False, eps=1e-5, momentum=0.1, peer_memory=True):
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.fuse_relu = fuse_relu
        self.torch_channels_last = torch_channels_last
        self.multi_stream = multi_stream
        self.max_cta_per_sm = max_cta_per_sm
        self.cta_launch_margin = cta_launch_margin
        self.bn_group = bn_group
        self.process_group = None
        if bn_group > 1:
            self.process_group = _bn_group(bn_group)
            if peer_memory and torch.cuda.is_available():
                # statistics exchanged through hipIpc peer buffers over xGMI (the reference's
                # groupbn IPC design, parallel/peer_memory.py) instead of one RCCL call per layer
                from ...parallel.peer_memory import enable_peer_memory

                enable_peer_memory(self.process_group)

    def synchronize_over(self, process_group=None, peer_memory=True):
        """Share the training statistics over ``process_group`` (None = every rank) — what
        ``apex.parallel.convert_syncbn_model`` does to this module.  Collective when peer memory
        is enabled (every member must call it in the same order)."""
        import torch.distributed as dist

        self.process_group = process_group
        self.bn_group = dist.get_world_size(process_group)
        if self.bn_group > 1 and peer_memory and torch.cuda.is_available():
            from ...parallel.peer_memory import enable_peer_memory

            enable_peer_memory(self.process_group)
        return self

    def _check_input_dim(self, input):
        if input.dim() != 4:
            raise ValueError("expected 4D input (got {}D input)".format(input.dim()))

    def forward(self, x, z=None, fork=False):
        if z is not None:
            assert self.fuse_relu, "BatchNorm2d_NHWC: z (residual) requires fuse_relu=True"
        training = self.training or not self.track_running_stats
        if self.bn_group > 1 and training:
            c = x.size(1) if (self.torch_channels_last and x.dim() == 4) else x.size(-1)
            if (_native.use_native(x) and c % 8 == 0 and self.weight is not None
                    and self.weight.dtype == torch.float32):
                return _BnNHWCGroupFunction.apply(x, z, self.weight, self.bias, self.running_mean, self.running_var,
                                                  self.momentum, self.eps, self.fuse_relu, self.process_group,
                                                  self.torch_channels_last, fork)
            from ...parallel.optimized_sync_batchnorm import SyncBatchnormFunction

            xv = x.permute(0, 2, 3, 1) if self.torch_channels_last else x
            zv = (z.permute(0, 2, 3, 1) if self.torch_channels_last else z) if z is not None else None
            y = SyncBatchnormFunction.apply(xv, zv, self.weight, self.bias, self.running_mean, self.running_var,
                                            self.eps, True, self.momentum, self.process_group, True, self.fuse_relu)
            y = y.permute(0, 3, 1, 2) if self.torch_channels_last else y
            return (y, y) if fork else y
        return bn_nhwc_function(x, z, self.weight, self.bias, self.running_mean, self.running_var, self.momentum,
                                self.eps, self.fuse_relu, training, self.torch_channels_last, fork)


_GROUPS = {}


def _bn_group(bn_group):
    """RCCL sub-group of ``bn_group`` adjacent ranks containing this rank (created collectively)."""
    import torch.distributed as dist

    if bn_group in _GROUPS:
        return _GROUPS[bn_group]
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world >= bn_group and world % bn_group == 0, "world size must be a multiple of bn_group"
    mine = None
    for start in range(0, world, bn_group):
        g = dist.new_group(list(range(start, start + bn_group)))
        if start <= rank < start + bn_group:
            mine = g
    _GROUPS[bn_group] = mine
    return mine
