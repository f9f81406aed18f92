"""SyncBatchNorm (reference apex/parallel/optimized_sync_batchnorm.py:9-85 and
optimized_sync_batchnorm_kernel.py:7-119).

Forward: local Welford (mean, biased var) -> ONE all_gather of [mean | var | count] per layer ->
Welford merge -> normalize.  Backward: local (sum_dy, sum_dy_xmu, dgamma, dbeta) -> ONE
all_reduce of [sum_dy | sum_dy_xmu] -> dx.  Stats kernels are the gfx950 Welford kernels in
``csrc/syncbn``; the collectives are RCCL (latency-bound, 8C bytes per layer)."""
import torch
from torch.nn import functional as F
from torch.nn.modules.batchnorm import _BatchNorm

from .optimized_sync_batchnorm_kernel import SyncBatchnormFunction  # noqa: F401


class SyncBatchNorm(_BatchNorm):
    """Batch norm whose training statistics are reduced across ``process_group``.

    ``channel_last=True`` takes the channel as the last dim (NHWC); ``fuse_relu`` / ``z`` fuse a
    residual add + ReLU into the normalization (channel_last only, as in the reference)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None, channel_last=False, fuse_relu=False):
        super(SyncBatchNorm, self).__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                                            track_running_stats=track_running_stats)
        self.process_group = process_group
        self.channel_last = channel_last
        self.fuse_relu = fuse_relu

    def _specify_process_group(self, process_group):
        self.process_group = process_group

    def _specify_channel_last(self, channel_last):
        self.channel_last = channel_last

    def _check_input_dim(self, input):
        if input.dim() < 2:
            raise ValueError("expected at least 2D input (got {}D input)".format(input.dim()))

    def _torch_channels_last(self, input):
        """True for an NCHW-shaped tensor in torch ``channels_last`` memory (what a channels_last
        convolution produces).  With ``channel_last=True`` the module also accepts an explicit
        NHWC tensor ([N, H, W, C], contiguous); the two are told apart by where ``num_features``
        sits and by the strides, so ``convert_syncbn_model(model, channel_last=True)`` on a
        channels_last model works."""
        if input.dim() != 4 or input.size(1) != self.num_features:
            return False
        if not input.is_contiguous(memory_format=torch.channels_last):
            return False
        if not input.is_contiguous():
            return True
        # both layouts are dense (e.g. H = W = 1): only an explicit-NHWC request whose last dim
        # really is the channel dim keeps the NHWC reading
        return not (self.channel_last and input.size(-1) == self.num_features)

    def forward(self, input, z=None):
        self._check_input_dim(input)
        if self._torch_channels_last(input):
            # torch channels_last memory: run the c_last kernels on a zero-copy NHWC view and
            # hand back an NCHW-shaped, channels_last-strided result
            zv = z.permute(0, 2, 3, 1) if z is not None else None
            out = self._forward_impl(input.permute(0, 2, 3, 1), zv, True)
            return out.permute(0, 3, 1, 2)
        channel_last = self.channel_last if input.dim() != 2 else True
        return self._forward_impl(input, z, channel_last)

    def _forward_impl(self, input, z, channel_last):
        if (not self.training and self.track_running_stats and not channel_last and not self.fuse_relu
                and z is None):
            return F.batch_norm(input, self.running_mean, self.running_var, self.weight, self.bias, False, 0.0,
                                self.eps)
        factor = 0.0
        if self.training and self.track_running_stats:
            self.num_batches_tracked += 1
            factor = 1.0 / float(self.num_batches_tracked) if self.momentum is None else self.momentum
        return SyncBatchnormFunction.apply(input, z, self.weight, self.bias, self.running_mean, self.running_var,
                                           self.eps, self.training or not self.track_running_stats, factor,
                                           self.process_group, channel_last, self.fuse_relu)
