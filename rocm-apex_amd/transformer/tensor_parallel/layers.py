"""Tensor-parallel layers (reference apex/transformer/tensor_parallel/layers.py:44-477).

* ``VocabParallelEmbedding`` — vocabulary sharded over the TP group; out-of-shard tokens are
  masked to zero and the partial embeddings summed with one all-reduce.
* ``ColumnParallelLinear`` — output features sharded (Y_i = X A_i); in backward the grad-input
  all-reduce is issued asynchronously and overlapped with the weight-gradient GEMM
  (reference :206-240).  Optional ``gather_output``.
* ``RowParallelLinear`` — input features sharded; partial outputs summed with one all-reduce.

MI355X additions: ``sequence_parallel_enabled`` (activations between TP regions kept 1/tp along
the sequence; the all-reduces become reduce-scatter / all-gather pairs of the same xGMI volume),
and the GEMM + bias epilogue goes through :mod:`apex.fused_dense` (gfx950 MFMA kernel) when it
supports the dtype, else ``torch.matmul`` (hipBLASLt).
"""
import os

import torch
import torch.nn.functional as F
from torch.nn import init
from torch.nn.parameter import Parameter

from ..._autocast_utils import _autocast_disabled, _cast_if_autocast_enabled
from ..parallel_state import get_tensor_model_parallel_group, get_tensor_model_parallel_rank, \
    get_tensor_model_parallel_world_size
from ..utils import divide
from .mappings import (_gather_along_first_dim, _reduce_scatter_along_first_dim,
                       copy_to_tensor_model_parallel_region, gather_from_tensor_model_parallel_region,
                       reduce_from_tensor_model_parallel_region, reduce_scatter_to_sequence_parallel_region,
                       scatter_to_tensor_model_parallel_region)
from .random import get_cuda_rng_tracker
from .utils import VocabUtility

_MODEL_PARALLEL_ATTRIBUTE_DEFAULTS = {"tensor_model_parallel": False, "partition_dim": -1, "partition_stride": 1}


def param_is_not_tensor_parallel_duplicate(param):
    return (hasattr(param, "tensor_model_parallel") and param.tensor_model_parallel) or (
        get_tensor_model_parallel_rank() == 0)


def set_tensor_model_parallel_attributes(tensor, is_parallel, dim, stride):
    for attribute in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        assert not hasattr(tensor, attribute)
    setattr(tensor, "tensor_model_parallel", is_parallel)
    setattr(tensor, "partition_dim", dim)
    setattr(tensor, "partition_stride", stride)


def set_defaults_if_not_set_tensor_model_parallel_attributes(tensor):
    for attribute, value in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS.items():
        if not hasattr(tensor, attribute):
            setattr(tensor, attribute, value)


def copy_tensor_model_parallel_attributes(destination_tensor, source_tensor):
    for attribute in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        if hasattr(source_tensor, attribute):
            setattr(destination_tensor, attribute, getattr(source_tensor, attribute))


def _default_device():
    return torch.cuda.current_device() if torch.cuda.is_available() else "cpu"


def _initialize_affine_weight_gpu(weight, init_method, partition_dim, stride=1):
    """Initialise this rank's shard directly on the device under the TP RNG stream."""
    set_tensor_model_parallel_attributes(tensor=weight, is_parallel=True, dim=partition_dim, stride=stride)
    with get_cuda_rng_tracker().fork():
        init_method(weight)


def _initialize_affine_weight_cpu(weight, output_size, input_size, per_partition_size, partition_dim, init_method,
                                  stride=1, return_master_weight=False, *, params_dtype=torch.float32):
    """Build the full master weight on every rank (CPU, fp32), keep this rank's strided shard."""
    set_tensor_model_parallel_attributes(tensor=weight, is_parallel=True, dim=partition_dim, stride=stride)
    master_weight = torch.empty(output_size, input_size, dtype=torch.float, requires_grad=False)
    init_method(master_weight)
    master_weight = master_weight.to(dtype=params_dtype)
    per_partition_per_stride_size = divide(per_partition_size, stride)
    weight_list = torch.split(master_weight, per_partition_per_stride_size, dim=partition_dim)
    rank = get_tensor_model_parallel_rank()
    world_size = get_tensor_model_parallel_world_size()
    my_weight_list = weight_list[rank::world_size]
    with torch.no_grad():
        weight.copy_(torch.cat(my_weight_list, dim=partition_dim).to(weight.device))
    if return_master_weight:
        return master_weight
    return None


def _sync_lt_picks(problem):
    """Rank 0's hipBLASLt picks for the tensor-parallel group (fused_dense.maybe_sync_lt_plans) the
    first time this TP problem runs; True when the caller must re-run the GEMM on the agreed pick."""
    from .. import parallel_state as ps

    if ps._TENSOR_MODEL_PARALLEL_GROUP is None:
        return False
    from ...fused_dense.fused_dense import maybe_sync_lt_plans

    return maybe_sync_lt_plans(ps._TENSOR_MODEL_PARALLEL_GROUP, problem)


def _linear(x, weight, bias):
    """y = x W^T + b on fused_dense's route: the hipBLASLt bias-epilogue GEMM with per-shape timed
    plans by default (APEX_AMD_DENSE_ROUTE=lt: 87-97 vs 124 us for the native kernel at the GPT-2
    QKV shape 16384 x 3072 x 1024, 31 vs 41 us at 1024 x 1024; profiles/gemm_routes_r04t.jsonl),
    the native GEMM + bias kernel with APEX_AMD_DENSE_ROUTE=native, torch elsewhere."""
    try:
        from ...fused_dense import fused_dense as fd
    except Exception:  # pragma: no cover - module not importable
        fd = None
    route = os.environ.get("APEX_AMD_TP_LINEAR", "")  # lt | torch | native (A/B override)
    if fd is not None and fd.fused_linear_available(x, weight, bias) and route != "torch":
        if route == "native" or (not route and fd.route_mode() == "native"):
            return fd.linear_bias_forward(x, weight, bias)
        y = fd._lib_dense_fwd(x, weight, bias)
        # one algorithm per GEMM across the tensor-parallel group: the first call of a problem
        # syncs rank 0's pick and recomputes, so even that call's output is rank-consistent
        if _sync_lt_picks(("fwd", x.numel() // x.shape[-1], weight.shape[0], weight.shape[1], str(x.dtype),
                           bias is not None)):
            y = fd._lib_dense_fwd(x, weight, bias)
        return y
    if bias is not None and x.dim() >= 2:
        return torch.addmm(bias, x.reshape(-1, x.shape[-1]), weight.t()).view(x.shape[:-1] + (weight.shape[0],))
    out = torch.matmul(x, weight.t())
    return out + bias if bias is not None else out


from ... import _native  # noqa: E402


def _wgrad(go2, ti2):
    """dW[N, K] = go2[M, N]^T ti2[M, K]: fused_dense.wgrad_gemm (the native split-K MFMA kernel for
    small N x K outputs, e.g. the 1024 x 1024 attention projection at 16k tokens: 64 vs 108 us;
    hipBLASLt with per-shape top-8 timing otherwise, e.g. the QKV 3072 x 1024: 149 vs 176 us;
    profiles/gemm_routes_r04t.jsonl)."""
    if go2.is_cuda:
        from ...fused_dense.fused_dense import wgrad_gemm

        dw = wgrad_gemm(go2, ti2)
        if _sync_lt_picks(("wgrad", go2.shape[0], go2.shape[1], ti2.shape[1], str(go2.dtype))):
            dw = wgrad_gemm(go2, ti2)
        return dw
    return go2.t().matmul(ti2)


class VocabParallelEmbedding(torch.nn.Module):
    """Embedding parallelized in the vocabulary dimension."""

    def __init__(self, num_embeddings, embedding_dim, init_method=init.xavier_normal_, *, params_dtype=torch.float32,
                 use_cpu_initialization=False):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.padding_idx = None
        self.max_norm = None
        self.norm_type = 2.0
        self.scale_grad_by_freq = False
        self.sparse = False
        self._weight = None
        self.tensor_model_parallel_size = get_tensor_model_parallel_world_size()
        self.vocab_start_index, self.vocab_end_index = VocabUtility.vocab_range_from_global_vocab_size(
            self.num_embeddings, get_tensor_model_parallel_rank(), self.tensor_model_parallel_size)
        self.num_embeddings_per_partition = self.vocab_end_index - self.vocab_start_index
        if use_cpu_initialization or not torch.cuda.is_available():
            self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, self.embedding_dim,
                                                dtype=params_dtype, device=None if use_cpu_initialization
                                                else _default_device()))
            _initialize_affine_weight_cpu(self.weight, self.num_embeddings, self.embedding_dim,
                                          self.num_embeddings_per_partition, 0, init_method, params_dtype=params_dtype)
        else:
            self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, self.embedding_dim,
                                                device=_default_device(), dtype=params_dtype))
            _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=0, stride=1)

    def forward(self, input_):
        if self.tensor_model_parallel_size > 1:
            input_mask = (input_ < self.vocab_start_index) | (input_ >= self.vocab_end_index)
            masked_input = input_.clone() - self.vocab_start_index
            masked_input[input_mask] = 0
        else:
            masked_input = input_
        output_parallel = F.embedding(masked_input, self.weight, self.padding_idx, self.max_norm, self.norm_type,
                                      self.scale_grad_by_freq, self.sparse)
        if self.tensor_model_parallel_size > 1:
            output_parallel[input_mask, :] = 0.0
        return reduce_from_tensor_model_parallel_region(output_parallel)


class LinearWithGradAccumulationAndAsyncCommunication(torch.autograd.Function):
    """Linear whose backward overlaps the TP grad-input collective with the wgrad GEMM.

    async_grad_allreduce: grad_input all-reduce (ColumnParallel, reference :206-234).
    sequence_parallel:    input all-gathered along dim 0 in forward; grad_input reduce-scattered
                          in backward (overlapped the same way)."""

    @staticmethod
    def forward(ctx, input, weight, bias, async_grad_allreduce, sequence_parallel):
        ctx.use_bias = bias is not None
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.sequence_parallel = sequence_parallel
        total_input = _gather_along_first_dim(input) if sequence_parallel else input
        ctx.save_for_backward(input, weight)
        return _linear(total_input, weight, bias)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        total_input = _gather_along_first_dim(input) if ctx.sequence_parallel else input
        grad_input = grad_output.matmul(weight)
        handle = None
        group = get_tensor_model_parallel_group()
        if ctx.sequence_parallel:
            gi = grad_input.contiguous()
            sub = torch.empty((gi.shape[0] // get_tensor_model_parallel_world_size(),) + tuple(gi.shape[1:]),
                              dtype=gi.dtype, device=gi.device)
            handle = torch.distributed.reduce_scatter_tensor(sub, gi, group=group, async_op=True)
        elif ctx.async_grad_allreduce:
            handle = torch.distributed.all_reduce(grad_input, group=group, async_op=True)
        go2 = grad_output.reshape(-1, grad_output.shape[-1])
        ti2 = total_input.reshape(-1, total_input.shape[-1])
        grad_weight = _wgrad(go2, ti2)
        grad_bias = _native.column_sum(go2, go2.dtype) if ctx.use_bias else None
        if handle is not None:
            handle.wait()
        if ctx.sequence_parallel:
            grad_input = sub
        return grad_input, grad_weight, grad_bias, None, None


def linear_with_grad_accumulation_and_async_allreduce(input, weight, bias, async_grad_allreduce,
                                                      sequence_parallel_enabled=False):
    args = _cast_if_autocast_enabled(input, weight, bias, async_grad_allreduce, sequence_parallel_enabled)
    with _autocast_disabled():
        return LinearWithGradAccumulationAndAsyncCommunication.apply(*args)


def column_parallel_linear(input, weight, bias):
    """Reference name (:237): async grad all-reduce variant."""
    return linear_with_grad_accumulation_and_async_allreduce(input, weight, bias, True, False)


ColumnParallelLinearWithAsyncAllreduce = LinearWithGradAccumulationAndAsyncCommunication


class ColumnParallelLinear(torch.nn.Module):
    """Y = X A + b with A split along its output dimension: A = [A_1, ..., A_p].

    Returns ``(output, output_bias)`` — ``output_bias`` is the bias when ``skip_bias_add``."""

    def __init__(self, input_size, output_size, bias=True, gather_output=True, init_method=init.xavier_normal_,
                 stride=1, keep_master_weight_for_test=False, skip_bias_add=False, *,
                 no_async_tensor_model_parallel_allreduce=False, params_dtype=torch.float32,
                 use_cpu_initialization=False, sequence_parallel_enabled=False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.gather_output = gather_output
        world_size = get_tensor_model_parallel_world_size()
        self.output_size_per_partition = divide(output_size, world_size)
        self.skip_bias_add = skip_bias_add
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if sequence_parallel_enabled and gather_output:
            raise RuntimeError("sequence_parallel_enabled requires gather_output=False")
        cpu_init = use_cpu_initialization or not torch.cuda.is_available()
        dev = None if use_cpu_initialization else _default_device()
        self.weight = Parameter(torch.empty(self.output_size_per_partition, self.input_size, dtype=params_dtype,
                                            device=dev))
        if cpu_init:
            self.master_weight = _initialize_affine_weight_cpu(self.weight, self.output_size, self.input_size,
                                                               self.output_size_per_partition, 0, init_method,
                                                               stride=stride,
                                                               return_master_weight=keep_master_weight_for_test,
                                                               params_dtype=params_dtype)
        else:
            _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=0, stride=stride)
        if bias:
            self.bias = Parameter(torch.empty(self.output_size_per_partition, dtype=params_dtype, device=dev))
            set_tensor_model_parallel_attributes(self.bias, True, 0, stride)
            with torch.no_grad():
                self.bias.zero_()
        else:
            self.register_parameter("bias", None)
        self.async_tensor_model_parallel_allreduce = (not no_async_tensor_model_parallel_allreduce
                                                      and world_size > 1 and not sequence_parallel_enabled)

    def forward(self, input_):
        bias = self.bias if not self.skip_bias_add else None
        if self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled:
            input_parallel = input_
        else:
            input_parallel = copy_to_tensor_model_parallel_region(input_)
        output_parallel = linear_with_grad_accumulation_and_async_allreduce(
            input_parallel, self.weight, bias, self.async_tensor_model_parallel_allreduce,
            self.sequence_parallel_enabled)
        output = gather_from_tensor_model_parallel_region(output_parallel) if self.gather_output else output_parallel
        output_bias = self.bias if self.skip_bias_add else None
        return output, output_bias


class RowParallelLinear(torch.nn.Module):
    """Y = X A + b with A split along its input dimension and X along its last dimension.

    Returns ``(output, output_bias)``; the bias is not parallelized."""

    def __init__(self, input_size, output_size, bias=True, input_is_parallel=False, init_method=init.xavier_normal_,
                 stride=1, keep_master_weight_for_test=False, skip_bias_add=False, *, params_dtype=torch.float32,
                 use_cpu_initialization=False, sequence_parallel_enabled=False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.input_is_parallel = input_is_parallel
        world_size = get_tensor_model_parallel_world_size()
        self.input_size_per_partition = divide(input_size, world_size)
        self.skip_bias_add = skip_bias_add
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if sequence_parallel_enabled and not input_is_parallel:
            raise RuntimeError("To enable `sequence_parallel_enabled`, `input_is_parallel` must be `True`")
        cpu_init = use_cpu_initialization or not torch.cuda.is_available()
        dev = None if use_cpu_initialization else _default_device()
        self.weight = Parameter(torch.empty(self.output_size, self.input_size_per_partition, dtype=params_dtype,
                                            device=dev))
        if cpu_init:
            self.master_weight = _initialize_affine_weight_cpu(self.weight, self.output_size, self.input_size,
                                                               self.input_size_per_partition, 1, init_method,
                                                               stride=stride,
                                                               return_master_weight=keep_master_weight_for_test,
                                                               params_dtype=params_dtype)
        else:
            _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=1, stride=stride)
        if bias:
            self.bias = Parameter(torch.empty(self.output_size, dtype=params_dtype, device=dev))
            setattr(self.bias, "sequence_parallel_enabled", sequence_parallel_enabled)
            with torch.no_grad():
                self.bias.zero_()
        else:
            self.register_parameter("bias", None)

    def forward(self, input_):
        input_parallel = input_ if self.input_is_parallel else scatter_to_tensor_model_parallel_region(input_)
        output_parallel = linear_with_grad_accumulation_and_async_allreduce(input_parallel, self.weight, None, False,
                                                                            False)
        if self.sequence_parallel_enabled:
            output_ = reduce_scatter_to_sequence_parallel_region(output_parallel)
        else:
            output_ = reduce_from_tensor_model_parallel_region(output_parallel)
        if not self.skip_bias_add:
            output = output_ + self.bias if self.bias is not None else output_
            output_bias = None
        else:
            output = output_
            output_bias = self.bias
        return output, output_bias


__all__ = ["VocabParallelEmbedding", "ColumnParallelLinear", "RowParallelLinear",
           "set_tensor_model_parallel_attributes", "set_defaults_if_not_set_tensor_model_parallel_attributes",
           "copy_tensor_model_parallel_attributes", "param_is_not_tensor_parallel_duplicate",
           "linear_with_grad_accumulation_and_async_allreduce", "column_parallel_linear",
           "_reduce_scatter_along_first_dim"]
