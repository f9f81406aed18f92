"""Model parallel utility interface (reference apex/transformer/tensor_parallel/__init__.py)."""
from .cross_entropy import vocab_parallel_cross_entropy
from .data import broadcast_data
from .layers import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,
                     copy_tensor_model_parallel_attributes, param_is_not_tensor_parallel_duplicate,
                     set_defaults_if_not_set_tensor_model_parallel_attributes, set_tensor_model_parallel_attributes,
                     linear_with_grad_accumulation_and_async_allreduce)
from .mappings import (copy_to_tensor_model_parallel_region, gather_from_sequence_parallel_region,
                       gather_from_tensor_model_parallel_region, reduce_from_tensor_model_parallel_region,
                       reduce_scatter_to_sequence_parallel_region, scatter_to_sequence_parallel_region,
                       scatter_to_tensor_model_parallel_region)
from .memory import MemoryBuffer, RingMemBuffer, allocate_mem_buff, get_mem_buff
from .random import (CounterRNGStreams, CudaRNGStatesTracker, checkpoint, get_counter_rng_streams, get_cuda_rng_tracker, init_checkpointed_activations_memory_buffer,
                     model_parallel_cuda_manual_seed, reset_checkpointed_activations_memory_buffer)
from .utils import VocabUtility, split_tensor_along_last_dim

__all__ = [
    "CounterRNGStreams", "get_counter_rng_streams",
    "vocab_parallel_cross_entropy", "broadcast_data", "ColumnParallelLinear", "RowParallelLinear",
    "VocabParallelEmbedding", "set_tensor_model_parallel_attributes",
    "set_defaults_if_not_set_tensor_model_parallel_attributes", "copy_tensor_model_parallel_attributes",
    "copy_to_tensor_model_parallel_region", "gather_from_tensor_model_parallel_region",
    "reduce_from_tensor_model_parallel_region", "scatter_to_tensor_model_parallel_region", "checkpoint",
    "get_cuda_rng_tracker", "init_checkpointed_activations_memory_buffer", "model_parallel_cuda_manual_seed",
    "reset_checkpointed_activations_memory_buffer", "split_tensor_along_last_dim",
]
