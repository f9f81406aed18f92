"""Autograd-aware tensor-parallel collectives (reference apex/transformer/tensor_parallel/mappings.py:23-159).

=========================  =====================  ======================
function                   forward                backward
=========================  =====================  ======================
copy_to_...                identity               all-reduce (TP)
reduce_from_...            all-reduce (TP)        identity
scatter_to_...             split last dim         all-gather last dim
gather_from_...            all-gather last dim    split last dim
scatter_to_sequence_...    split first dim        all-gather first dim
gather_from_sequence_...   all-gather first dim   reduce-scatter first dim
reduce_scatter_to_seq...   reduce-scatter dim 0   all-gather first dim
=========================  =====================  ======================

All gathers go through ``all_gather_into_tensor`` into one contiguous buffer (one RCCL call, no
per-rank list); the last-dim gather then interleaves with a single ``cat``.  The sequence-parallel
(first-dim) variants are an MI355X addition — the reference has no sequence parallelism — and
turn each TP all-reduce into a reduce-scatter + all-gather pair that moves the same bytes over
xGMI while keeping activations 1/tp-sized between them.
"""
import torch

from ..parallel_state import get_tensor_model_parallel_group, get_tensor_model_parallel_rank, \
    get_tensor_model_parallel_world_size
from .utils import split_tensor_along_last_dim


def _reduce(input_):
    if get_tensor_model_parallel_world_size() == 1:
        return input_
    torch.distributed.all_reduce(input_, group=get_tensor_model_parallel_group())
    return input_


def _split_along_last_dim(input_):
    world_size = get_tensor_model_parallel_world_size()
    if world_size == 1:
        return input_
    input_list = split_tensor_along_last_dim(input_, world_size)
    return input_list[get_tensor_model_parallel_rank()].contiguous()


def _split_along_first_dim(input_):
    world_size = get_tensor_model_parallel_world_size()
    if world_size == 1:
        return input_
    n = input_.size(0)
    assert n % world_size == 0, "first dimension must be divisible by the tensor parallel size"
    local = n // world_size
    rank = get_tensor_model_parallel_rank()
    return input_[rank * local:(rank + 1) * local].contiguous()


def _gather_along_last_dim(input_):
    world_size = get_tensor_model_parallel_world_size()
    if world_size == 1:
        return input_
    x = input_.contiguous()
    buf = torch.empty(world_size * x.numel(), dtype=x.dtype, device=x.device)
    torch.distributed.all_gather_into_tensor(buf, x.view(-1), group=get_tensor_model_parallel_group())
    return torch.cat(buf.view((world_size,) + tuple(x.shape)).unbind(0), dim=-1).contiguous()


def _gather_along_first_dim(input_):
    world_size = get_tensor_model_parallel_world_size()
    if world_size == 1:
        return input_
    x = input_.contiguous()
    out = torch.empty((world_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    torch.distributed.all_gather_into_tensor(out, x, group=get_tensor_model_parallel_group())
    return out


def _reduce_scatter_along_first_dim(input_):
    world_size = get_tensor_model_parallel_world_size()
    if world_size == 1:
        return input_
    x = input_.contiguous()
    assert x.shape[0] % world_size == 0
    out = torch.empty((x.shape[0] // world_size,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    torch.distributed.reduce_scatter_tensor(out, x, group=get_tensor_model_parallel_group())
    return out


class _CopyToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def symbolic(graph, input_):
        return input_

    @staticmethod
    def forward(ctx, input_):
        return input_

    @staticmethod
    def backward(ctx, grad_output):
        return _reduce(grad_output)


class _ReduceFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def symbolic(graph, input_):
        return _reduce(input_)

    @staticmethod
    def forward(ctx, input_):
        return _reduce(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class _ScatterToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def symbolic(graph, input_):
        return _split_along_last_dim(input_)

    @staticmethod
    def forward(ctx, input_):
        return _split_along_last_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_last_dim(grad_output)


class _GatherFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def symbolic(graph, input_):
        return _gather_along_last_dim(input_)

    @staticmethod
    def forward(ctx, input_):
        return _gather_along_last_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _split_along_last_dim(grad_output)


class _ScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _split_along_first_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_first_dim(grad_output)


class _GatherFromSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_, to_model_parallel=True):
        ctx.to_model_parallel = to_model_parallel
        return _gather_along_first_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.to_model_parallel:
            return _reduce_scatter_along_first_dim(grad_output), None
        return _split_along_first_dim(grad_output), None


class _ReduceScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _reduce_scatter_along_first_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_first_dim(grad_output)


def copy_to_tensor_model_parallel_region(input_):
    return _CopyToModelParallelRegion.apply(input_)


def reduce_from_tensor_model_parallel_region(input_):
    return _ReduceFromModelParallelRegion.apply(input_)


def scatter_to_tensor_model_parallel_region(input_):
    return _ScatterToModelParallelRegion.apply(input_)


def gather_from_tensor_model_parallel_region(input_):
    return _GatherFromModelParallelRegion.apply(input_)


def scatter_to_sequence_parallel_region(input_):
    return _ScatterToSequenceParallelRegion.apply(input_)


def gather_from_sequence_parallel_region(input_, to_model_parallel=True):
    return _GatherFromSequenceParallelRegion.apply(input_, to_model_parallel)


def reduce_scatter_to_sequence_parallel_region(input_):
    return _ReduceScatterToSequenceParallelRegion.apply(input_)
