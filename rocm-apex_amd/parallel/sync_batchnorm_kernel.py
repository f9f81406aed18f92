"""SyncBatchnormFunction of the pure-PyTorch SyncBatchNorm (reference
apex/parallel/sync_batchnorm_kernel.py:7-87): all-reduces of the per-channel mean and mean of
squares in forward, of the gradient sums in backward."""
import torch
import torch.distributed as dist
from torch.autograd.function import Function


class SyncBatchnormFunction(Function):
    @staticmethod
    def forward(ctx, input, weight, bias, running_mean, running_var, eps, process_group, world_size):
        c = input.size(1)
        x = input.transpose(0, 1).contiguous().view(c, -1).float()
        mean = x.mean(1)
        sqr_mean = (x * x).mean(1)
        if world_size > 1:
            dist.all_reduce(mean, dist.ReduceOp.SUM, process_group)
            dist.all_reduce(sqr_mean, dist.ReduceOp.SUM, process_group)
            mean /= world_size
            sqr_mean /= world_size
        var = sqr_mean - mean * mean
        n = x.size(1) * world_size
        inv_std = torch.rsqrt(var + eps)
        ctx.save_for_backward(input, weight, mean, inv_std)
        ctx.process_group = process_group
        ctx.world_size = world_size
        shp = (1, -1) + (1,) * (input.dim() - 2)
        y = (input.float() - mean.view(shp)) * inv_std.view(shp)
        if weight is not None:
            y = y * weight.float().view(shp) + bias.float().view(shp)
        ctx.unbiased_var = var * n / max(n - 1, 1)
        return y.to(input.dtype)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight, mean, inv_std = ctx.saved_tensors
        c = input.size(1)
        shp = (1, -1) + (1,) * (input.dim() - 2)
        dy = grad_output.float()
        xmu = input.float() - mean.view(shp)
        red = tuple(d for d in range(input.dim()) if d != 1)
        mean_dy = dy.mean(red)
        mean_dy_xmu = (dy * xmu).mean(red)
        grad_weight = (dy * xmu * inv_std.view(shp)).sum(red) if weight is not None else None
        grad_bias = dy.sum(red) if weight is not None else None
        if ctx.world_size > 1:
            dist.all_reduce(mean_dy, dist.ReduceOp.SUM, ctx.process_group)
            dist.all_reduce(mean_dy_xmu, dist.ReduceOp.SUM, ctx.process_group)
            mean_dy /= ctx.world_size
            mean_dy_xmu /= ctx.world_size
        w = weight.float().view(shp) if weight is not None else 1.0
        dx = (dy - mean_dy.view(shp) - xmu * inv_std.view(shp) ** 2 * mean_dy_xmu.view(shp)) * inv_std.view(shp) * w
        return dx.to(input.dtype), grad_weight, grad_bias, None, None, None, None, None
