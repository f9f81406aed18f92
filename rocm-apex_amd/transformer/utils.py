"""Helpers shared by ``tensor_parallel`` and ``pipeline_parallel`` (reference apex/transformer/utils.py:8-36)."""
import torch


def ensure_divisibility(numerator, denominator):
    """Ensure that numerator is divisible by the denominator."""
    assert numerator % denominator == 0, "{} is not divisible by {}".format(numerator, denominator)


def divide(numerator, denominator):
    """Ensure that numerator is divisible by the denominator and return the division value."""
    ensure_divisibility(numerator, denominator)
    return numerator // denominator


def comm_device():
    """Device collectives run on: the current GPU under RCCL, the CPU under gloo (test tier)."""
    if torch.cuda.is_available() and torch.distributed.is_initialized() and \
            torch.distributed.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    if torch.cuda.is_available() and not torch.distributed.is_initialized():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def split_tensor_into_1d_equal_chunks(tensor):
    """This rank's 1/tp slice of the flattened tensor."""
    from . import parallel_state

    data = tensor.view(-1)
    partition_size = torch.numel(data) // parallel_state.get_tensor_model_parallel_world_size()
    start_index = partition_size * parallel_state.get_tensor_model_parallel_rank()
    return data[start_index:start_index + partition_size]


def gather_split_1d_tensor(tensor):
    """Inverse of :func:`split_tensor_into_1d_equal_chunks`: one all-gather into a flat buffer."""
    from . import parallel_state

    world_size = parallel_state.get_tensor_model_parallel_world_size()
    numel = torch.numel(tensor)
    gathered = torch.empty(world_size * numel, dtype=tensor.dtype, device=tensor.device, requires_grad=False)
    torch.distributed.all_gather_into_tensor(gathered, tensor.contiguous().view(-1),
                                             group=parallel_state.get_tensor_model_parallel_group())
    return gathered
