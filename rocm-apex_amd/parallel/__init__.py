"""Data parallelism: DistributedDataParallel, Reducer, SyncBatchNorm, LARC
(reference apex/parallel/__init__.py:10-95)."""
import torch

ReduceOp = torch.distributed.ReduceOp

from .distributed import DistributedDataParallel, Reducer  # noqa: E402,F401
from .optimized_sync_batchnorm import SyncBatchNorm  # noqa: E402,F401
from .LARC import LARC  # noqa: E402,F401


def convert_syncbn_model(module, process_group=None, channel_last=False):
    """Recursively replace every ``_BatchNorm`` with :class:`SyncBatchNorm` (state copied).

    ``channel_last`` selects the explicit-NHWC reading for 4-D inputs whose last dim is the
    channel dim; NCHW-shaped tensors in torch ``channels_last`` memory are recognised either way.
    The fused NHWC batch norm (``apex.contrib.groupbn.BatchNorm2d_NHWC``, which carries fused
    ReLU / residual inputs) is kept and synchronized in place over ``process_group`` instead."""
    mod = module
    if isinstance(module, torch.nn.modules.instancenorm._InstanceNorm):
        return module
    from ..contrib.groupbn.batch_norm import BatchNorm2d_NHWC

    if isinstance(module, BatchNorm2d_NHWC):
        module.synchronize_over(process_group)
        for name, child in module.named_children():
            module.add_module(name, convert_syncbn_model(child, process_group, channel_last))
        return module
    if isinstance(module, torch.nn.modules.batchnorm._BatchNorm):
        mod = SyncBatchNorm(module.num_features, module.eps, module.momentum, module.affine,
                            module.track_running_stats, process_group, channel_last=channel_last)
        mod.running_mean = module.running_mean
        mod.running_var = module.running_var
        mod.num_batches_tracked = module.num_batches_tracked
        if module.affine:
            mod.weight.data = module.weight.data.clone().detach()
            mod.bias.data = module.bias.data.clone().detach()
        mod = mod.to(module.weight.device if module.affine else module.running_mean.device)
    for name, child in module.named_children():
        mod.add_module(name, convert_syncbn_model(child, process_group=process_group, channel_last=channel_last))
    del module
    return mod


def create_syncbn_process_group(group_size):
    """Process groups of ``group_size`` consecutive ranks; returns the caller's group
    (``None`` for group_size 0 = whole world)."""
    if group_size == 0:
        return None
    world_size = torch.distributed.get_world_size()
    assert world_size >= group_size
    assert world_size % group_size == 0
    group = None
    for group_num in range(world_size // group_size):
        ids = list(range(group_num * group_size, (group_num + 1) * group_size))
        cur = torch.distributed.new_group(ranks=ids)
        if torch.distributed.get_rank() // group_size == group_num:
            group = cur
    assert group is not None
    return group
from .peer_memory import PeerExchange, disable_peer_memory, enable_peer_memory, get_peer_exchange  # noqa: E402,F401
