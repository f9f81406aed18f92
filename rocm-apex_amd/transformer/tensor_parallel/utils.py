"""Tensor-parallel utilities (reference apex/transformer/tensor_parallel/utils.py:20-54)."""
import torch

from ..utils import divide


def split_tensor_along_last_dim(tensor, num_partitions, contiguous_split_chunks=False):
    """Split ``tensor`` into ``num_partitions`` equal chunks along its last dimension."""
    last_dim = tensor.dim() - 1
    last_dim_size = divide(tensor.size()[last_dim], num_partitions)
    tensor_list = torch.split(tensor, last_dim_size, dim=last_dim)
    if contiguous_split_chunks:
        return tuple(chunk.contiguous() for chunk in tensor_list)
    return tensor_list


class VocabUtility:
    """Vocabulary range [first, last) owned by ``rank`` when split into ``world_size`` chunks."""

    @staticmethod
    def vocab_range_from_per_partition_vocab_size(per_partition_vocab_size, rank, world_size):
        index_f = rank * per_partition_vocab_size
        return index_f, index_f + per_partition_vocab_size

    @staticmethod
    def vocab_range_from_global_vocab_size(global_vocab_size, rank, world_size):
        per_partition_vocab_size = divide(global_vocab_size, world_size)
        return VocabUtility.vocab_range_from_per_partition_vocab_size(per_partition_vocab_size, rank, world_size)
