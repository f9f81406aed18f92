"""Pure-PyTorch SyncBatchNorm (reference apex/parallel/sync_batchnorm.py:9-134): two all-reduces
of per-channel mean and mean-of-squares in forward, two in backward.  Kept for API parity; the
default ``apex.parallel.SyncBatchNorm`` is the Welford/RCCL one in optimized_sync_batchnorm."""
import torch
import torch.distributed as dist
from torch.nn import functional as F
from torch.nn.modules.batchnorm import _BatchNorm

from .sync_batchnorm_kernel import SyncBatchnormFunction  # noqa: F401


class SyncBatchNorm(_BatchNorm):
    warned = False

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None, channel_last=False):
        super(SyncBatchNorm, self).__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                                            track_running_stats=track_running_stats)
        self.process_group = process_group
        self.channel_last = channel_last

    def _specify_process_group(self, process_group):
        self.process_group = process_group

    def forward(self, input):
        torch.cuda.nvtx.range_push("sync_bn_fw_with_mean_var") if input.is_cuda else None
        if not self.training and self.track_running_stats:
            out = F.batch_norm(input, self.running_mean, self.running_var, self.weight, self.bias, False, 0.0,
                               self.eps)
        else:
            ws = dist.get_world_size(self.process_group) if (dist.is_available() and dist.is_initialized()) else 1
            x = input.transpose(1, -1) if self.channel_last else input
            out = SyncBatchnormFunction.apply(x, self.weight, self.bias, None, None, self.eps,
                                              self.process_group, ws)
            if self.training and self.track_running_stats:
                with torch.no_grad():
                    c = x.size(1)
                    xf = x.transpose(0, 1).reshape(c, -1).float()
                    m = xf.mean(1)
                    v = xf.var(1, unbiased=True)
                    if ws > 1:
                        dist.all_reduce(m, group=self.process_group)
                        dist.all_reduce(v, group=self.process_group)
                        m /= ws
                        v /= ws
                    self.num_batches_tracked += 1
                    mom = self.momentum if self.momentum is not None else 1.0 / float(self.num_batches_tracked)
                    self.running_mean.mul_(1 - mom).add_(mom * m.to(self.running_mean.dtype))
                    self.running_var.mul_(1 - mom).add_(mom * v.to(self.running_var.dtype))
            if self.channel_last:
                out = out.transpose(1, -1)
        torch.cuda.nvtx.range_pop() if input.is_cuda else None
        return out
