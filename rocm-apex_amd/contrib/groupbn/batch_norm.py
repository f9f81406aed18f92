"""NHWC batch norm with fused ReLU and fused residual add + ReLU
(reference apex/contrib/groupbn/batch_norm.py:24-260 — ``BatchNorm2d_NHWC``).

GPU path: the gfx950 fused pipeline in ``csrc/groupbn/bn_nhwc.hip`` (3 passes forward, 5
backward, ReLU mask recomputed in registers, deterministic partial reductions).  The module
accepts either a logical NHWC tensor ``[N, H, W, C]`` or — with ``torch_channels_last=True`` — an
NCHW-shaped tensor in ``torch.channels_last`` memory (what convolutions produce); both are handed
to the kernels as the same zero-copy ``[M, C]`` view and the output keeps the input's layout.

``bn_group > 1`` (statistics shared by groups of adjacent ranks; the reference does this through
CUDA-IPC peer memory and compiles it out on HIP): the per-rank (mean, var, count) and the backward
(sum_dy, sum_dy_xmu) are exchanged through hipIpc peer buffers over xGMI — one single-workgroup
push/flag-wait kernel per layer (``apex.parallel.peer_memory``) — or, with ``peer_memory=False``,
by an RCCL sub-group all-gather / all-reduce.  CPU tensors
and channel counts that are not a multiple of 8 use the generic SyncBatchNorm primitives.
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

    def _check_input_dim(self, input):
        if input.dim() != 4:
            raise ValueError("expected 4D input (got {}D input)".format(input.dim()))

    def forward(self, x, z=None, fork=False):
        if z is not None:
            assert self.fuse_relu, "BatchNorm2d_NHWC: z (residual) requires fuse_relu=True"
        training = self.training or not self.track_running_stats
        if self.bn_group > 1 and training:
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
