"""Broadcast a batch from TP-rank 0 to its tensor-parallel group
(reference apex/transformer/tensor_parallel/data.py:25-113).

Two collectives per call as in the reference (sizes, then one flat buffer of every key), but
the size table is an int64 tensor on the communication device built without per-key syncs."""
import torch

from ..parallel_state import get_tensor_model_parallel_group, get_tensor_model_parallel_rank, \
    get_tensor_model_parallel_src_rank
from ..utils import comm_device

_MAX_DATA_DIM = 5


def _check_data_types(keys, data, target_dtype):
    for key in keys:
        assert data[key].dtype == target_dtype, "{} has data type {} which is different than {}".format(
            key, data[key].dtype, target_dtype)


def _build_key_size_numel_dictionaries(keys, data):
    max_dim = _MAX_DATA_DIM
    sizes = [0 for _ in range(max_dim) for _ in keys]
    if get_tensor_model_parallel_rank() == 0:
        offset = 0
        for key in keys:
            assert data[key].dim() < max_dim, "you should increase MAX_DATA_DIM"
            for i, s in enumerate(data[key].size()):
                sizes[i + offset] = s
            offset += max_dim
    sizes_t = torch.tensor(sizes, dtype=torch.long, device=comm_device())
    torch.distributed.broadcast(sizes_t, get_tensor_model_parallel_src_rank(), group=get_tensor_model_parallel_group())
    sizes_cpu = sizes_t.cpu().tolist()
    key_size, key_numel, total_numel, offset = {}, {}, 0, 0
    for key in keys:
        size, numel, i = [], 1, 0
        while i < max_dim and sizes_cpu[offset + i] > 0:
            size.append(sizes_cpu[offset + i])
            numel *= sizes_cpu[offset + i]
            i += 1
        key_size[key] = size
        key_numel[key] = numel
        total_numel += numel
        offset += max_dim
    return key_size, key_numel, total_numel


def broadcast_data(keys, data, datatype):
    """Broadcast ``{key: tensor}`` (all of dtype ``datatype``) from the first rank of each
    tensor-parallel group; returns device tensors on every member."""
    key_size, key_numel, total_numel = _build_key_size_numel_dictionaries(keys, data)
    dev = comm_device()
    if get_tensor_model_parallel_rank() == 0:
        _check_data_types(keys, data, datatype)
        flatten_data = torch.cat([data[key].contiguous().view(-1) for key in keys], dim=0).to(dev)
    else:
        flatten_data = torch.empty(total_numel, device=dev, dtype=datatype)
    torch.distributed.broadcast(flatten_data, get_tensor_model_parallel_src_rank(),
                                group=get_tensor_model_parallel_group())
    output, offset = {}, 0
    for key in keys:
        output[key] = flatten_data.narrow(0, offset, key_numel[key]).view(key_size[key])
        offset += key_numel[key]
    return output
