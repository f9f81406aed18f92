"""SyncBatchnormFunction of the optimized SyncBatchNorm (reference
apex/parallel/optimized_sync_batchnorm_kernel.py:7-119): gfx950 Welford statistics, ONE all_gather of
[mean | var | count] per layer (hipIpc peer exchange over xGMI when enabled, else RCCL), Welford
merge, normalize; backward ONE all_reduce of [sum_dy | sum_dy_xmu]."""
import torch
import torch.distributed as dist
from torch.autograd.function import Function

from ..ops import batchnorm as bnops
from .peer_memory import get_peer_exchange


class SyncBatchnormFunction(Function):
    @staticmethod
    def forward(ctx, input, z, weight, bias, running_mean, running_variance, eps, track_running_stats=True,
                momentum=1.0, process_group=None, channel_last=False, fuse_relu=False):
        input = input.contiguous() if not channel_last else input
        if channel_last and not input.is_contiguous():
            input = input.contiguous()
        world_size = 0
        peer_used = False
        if track_running_stats:
            num_channels = input.size(-1) if channel_last else input.size(1)
            count = input.numel() // num_channels
            mean, var_biased = bnops.welford_mean_var(input, channel_last)
            if process_group != "local" and dist.is_available() and dist.is_initialized():
                pg = process_group if process_group else dist.group.WORLD
                world_size = dist.get_world_size(pg)
                count_t = torch.full((1,), float(count), dtype=mean.dtype, device=mean.device)
                combined = torch.cat([mean.view(-1), var_biased.view(-1), count_t], dim=0)
                peer = get_peer_exchange(process_group)
                if peer is not None:  # hipIpc exchange over xGMI (parallel/peer_memory.py)
                    gathered = peer.all_gather(combined).to(combined.dtype)
                    peer_used = True
                elif dist.get_backend(pg) == "nccl":
                    gathered = torch.empty(world_size * combined.numel(), dtype=combined.dtype,
                                           device=combined.device)
                    dist.all_gather_into_tensor(gathered, combined, group=pg)
                    gathered = gathered.view(world_size, -1)
                else:
                    parts = [torch.empty_like(combined) for _ in range(world_size)]
                    dist.all_gather(parts, combined, group=pg)
                    gathered = torch.stack(parts, 0)
                mean_all, var_all, count_all = torch.split(gathered, num_channels, dim=1)
                count_all = count_all.reshape(-1)
                mean, var, inv_std = bnops.welford_parallel(mean_all, var_all, count_all.to(torch.int32), eps)
            else:
                count_all = torch.tensor([count], dtype=torch.int32, device=mean.device)
                inv_std = 1.0 / torch.sqrt(var_biased + eps)
                var = var_biased * count / max(count - 1, 1)
            if count == 1 and world_size < 2:
                raise ValueError("Expected more than 1 value per channel when training, got input size{}".format(
                    input.size()))
            if running_mean is not None:
                r_m = mean if running_mean.dtype != torch.float16 else mean.half()
                r_v = var if running_variance.dtype != torch.float16 else var.half()
                if peer_used:
                    # a timed-out peer exchange poisons mean/var with NaN (the step is skipped by
                    # the loss scaler); keep the running statistics as they were, sync-free
                    keep = torch.isfinite(r_m) & torch.isfinite(r_v)
                    running_mean.data.copy_(torch.where(keep, running_mean.data * (1 - momentum) + momentum * r_m,
                                                        running_mean.data))
                    running_variance.data.copy_(torch.where(
                        keep, running_variance.data * (1 - momentum) + momentum * r_v, running_variance.data))
                else:
                    running_mean.data.mul_(1 - momentum).add_(momentum * r_m)
                    running_variance.data.mul_(1 - momentum).add_(momentum * r_v)
        else:
            mean = running_mean.data.float()
            inv_std = 1.0 / torch.sqrt(running_variance.data.float() + eps)
            count_all = torch.tensor([1], dtype=torch.int32, device=mean.device)
        ctx.save_for_backward(input, weight, mean, inv_std, z, bias, count_all.to(torch.int32))
        ctx.process_group = process_group
        ctx.channel_last = channel_last
        ctx.world_size = world_size
        ctx.fuse_relu = fuse_relu
        return bnops.batchnorm_forward(input, mean, inv_std, weight, bias, channel_last, z, fuse_relu)

    @staticmethod
    def backward(ctx, grad_output):
        grad_output = grad_output.contiguous()
        saved_input, weight, mean, inv_std, z, bias, count = ctx.saved_tensors
        channel_last = ctx.channel_last
        grad_input = grad_z = grad_weight = grad_bias = None
        relu = ctx.fuse_relu
        zz = z if isinstance(z, torch.Tensor) else None
        if relu and zz is not None and ctx.needs_input_grad[1]:
            # the residual branch needs the masked gradient itself: materialize it once
            grad_output = bnops.relu_backward(grad_output, saved_input, zz, mean, inv_std, weight, bias, channel_last)
            grad_z = grad_output
            relu = False
        elif zz is not None and ctx.needs_input_grad[1]:
            grad_z = grad_output.clone()
        # with `relu` still set, the kernels mask dy by the recomputed output in registers
        sum_dy, sum_dy_xmu, grad_weight, grad_bias = bnops.reduce_bn(grad_output, saved_input, mean, inv_std, weight,
                                                                     channel_last, zz, bias, relu)
        if ctx.needs_input_grad[0]:
            if dist.is_available() and dist.is_initialized() and ctx.world_size > 0:
                c = sum_dy.shape[0]
                combined = torch.cat([sum_dy, sum_dy_xmu], dim=0)
                peer = get_peer_exchange(ctx.process_group)
                if peer is not None:
                    combined = peer.all_reduce_sum(combined)
                else:
                    dist.all_reduce(combined, dist.ReduceOp.SUM, ctx.process_group, async_op=False)
                sum_dy, sum_dy_xmu = torch.split(combined, c)
            grad_input = bnops.batchnorm_backward(grad_output, saved_input, mean, inv_std, weight, sum_dy, sum_dy_xmu,
                                                  count, channel_last, zz, bias, relu)
        if weight is None or not ctx.needs_input_grad[2]:
            grad_weight = None
        if weight is None or not ctx.needs_input_grad[3]:
            grad_bias = None
        return grad_input, grad_z, grad_weight, grad_bias, None, None, None, None, None, None, None, None
