"""Model-parallel RNG state tracking and activation checkpointing
(reference apex/transformer/tensor_parallel/random.py:36-294).

Two RNG streams per process (Megatron scheme):
  * the default generator — identical across a TP group (dropout outside TP regions);
  * the tracked "model-parallel-rng" state — seeded ``seed + 2718 + tp_rank`` so every TP rank
    draws different dropout masks inside TP regions.
``checkpoint`` recomputes the forward in backward with the CPU, device and tracker RNG states
restored, so dropout masks match the original forward exactly.  The device generator is HIP on
MI355X; without a GPU (CPU test tier) the CPU generator plays that role.
"""
import contextlib

import torch
from torch.utils.checkpoint import detach_variable

from ..parallel_state import get_tensor_model_parallel_rank
from ..utils import gather_split_1d_tensor, split_tensor_into_1d_equal_chunks
from .memory import allocate_mem_buff

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"
_CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER = None


def init_checkpointed_activations_memory_buffer(micro_batch_size, max_position_embeddings, hidden_size, num_layers,
                                                tensor_model_parallel_size, checkpoint_num_layers, fp16):
    """One arena for the (1/tp-split) inputs of every checkpointed segment."""
    per_layer = micro_batch_size * max_position_embeddings * hidden_size // tensor_model_parallel_size
    assert num_layers % checkpoint_num_layers == 0, "number of layers is not divisible by checkpoint-num-layers"
    numel = per_layer * (num_layers // checkpoint_num_layers)
    dtype = torch.half if fp16 else torch.float
    global _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER
    assert _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER is None, "checkpointed activations memory buffer is already allocated."
    _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER = allocate_mem_buff("checkpointed activations", numel, dtype,
                                                                track_usage=False)


def reset_checkpointed_activations_memory_buffer():
    if _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER is not None:
        _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER.reset()


def _device_rng_available():
    return torch.cuda.is_available()


def _get_device_rng_state():
    return torch.cuda.get_rng_state() if _device_rng_available() else torch.get_rng_state()


def _set_device_rng_state(new_state, device=-1):
    """Set the device generator state without cloning it (the reference's ``_set_cuda_rng_state``)."""
    if not _device_rng_available():
        torch.set_rng_state(new_state)
        return
    if device == -1:
        idx = torch.cuda.current_device()
    elif isinstance(device, torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
    elif isinstance(device, str):
        d = torch.device(device)
        idx = d.index if d.index is not None else torch.cuda.current_device()
    else:
        idx = int(device)
    torch.cuda.default_generators[idx].set_state(new_state)


_set_cuda_rng_state = _set_device_rng_state


def _device_manual_seed(seed):
    if _device_rng_available():
        torch.cuda.manual_seed(seed)
    else:
        torch.manual_seed(seed)


class CudaRNGStatesTracker:
    """Named device-RNG states; ``fork(name)`` runs a block under that state and advances it."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = states

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception("seed {} already exists".format(seed))
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception("cuda rng state {} already exists".format(name))
        orig = _get_device_rng_state()
        _device_manual_seed(seed)
        self.states_[name] = _get_device_rng_state()
        _set_device_rng_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception("cuda rng state {} is not added".format(name))
        orig = _get_device_rng_state()
        _set_device_rng_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _get_device_rng_state()
            _set_device_rng_state(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


class CounterRNGStreams:
    """Call counters of the counter-hash dropout streams (flash-attention probability dropout, the
    fused bias-dropout-add): a dropout mask here is a pure function of (seed, stream offset,
    element index), so the offset IS the generator state.  CheckpointFunction saves and restores
    it with the device generator and the tracker states, so a recomputed segment draws exactly the
    masks of its original forward."""

    def __init__(self):
        self.counts = {}

    def next(self, name):
        c = self.counts.get(name, 0) + 1
        self.counts[name] = c
        return c

    def get_states(self):
        return dict(self.counts)

    def set_states(self, states):
        self.counts = dict(states)


_COUNTER_RNG_STREAMS = CounterRNGStreams()


def get_counter_rng_streams():
    return _COUNTER_RNG_STREAMS


def model_parallel_cuda_manual_seed(seed):
    """Seed the default stream with ``seed`` and the tracked TP stream with
    ``seed + 2718 + tp_rank`` (call after initialize_model_parallel)."""
    tensor_model_parallel_seed = seed + 2718 + get_tensor_model_parallel_rank()
    _CUDA_RNG_STATE_TRACKER.reset()
    _device_manual_seed(seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, tensor_model_parallel_seed)


class CheckpointFunction(torch.autograd.Function):
    """torch.utils.checkpoint with the device RNG and the model-parallel tracker states saved and
    restored around the recompute; optionally keeps only a 1/tp slice of the first input."""

    @staticmethod
    def forward(ctx, run_function, distribute_saved_activations, *args):
        ctx.run_function = run_function
        ctx.distribute_saved_activations = distribute_saved_activations
        ctx.fwd_cpu_rng_state = torch.get_rng_state()
        ctx.fwd_cuda_rng_state = _get_device_rng_state()
        ctx.fwd_cuda_rng_state_tracker = get_cuda_rng_tracker().get_states()
        ctx.fwd_counter_streams = _COUNTER_RNG_STREAMS.get_states()
        with torch.no_grad():
            outputs = run_function(*args)
        if distribute_saved_activations:
            ctx.input_0_shape = args[0].data.shape
            args[0].data = split_tensor_into_1d_equal_chunks(args[0].data)
            if _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER is not None:
                args[0].data = _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER.add(args[0].data)
        ctx.save_for_backward(*args)
        return outputs

    @staticmethod
    def backward(ctx, *args):
        if not torch.autograd._is_checkpoint_valid():
            raise RuntimeError("Checkpointing is not compatible with .grad(), please use .backward() if possible")
        inputs = ctx.saved_tensors
        if ctx.distribute_saved_activations:
            inputs[0].data = gather_split_1d_tensor(inputs[0].data).view(ctx.input_0_shape)
        bwd_cpu_rng_state = torch.get_rng_state()
        bwd_cuda_rng_state = _get_device_rng_state()
        bwd_cuda_rng_state_tracker = get_cuda_rng_tracker().get_states()
        torch.set_rng_state(ctx.fwd_cpu_rng_state)
        _set_device_rng_state(ctx.fwd_cuda_rng_state)
        get_cuda_rng_tracker().set_states(ctx.fwd_cuda_rng_state_tracker)
        bwd_counter_streams = _COUNTER_RNG_STREAMS.get_states()
        _COUNTER_RNG_STREAMS.set_states(ctx.fwd_counter_streams)
        detached_inputs = detach_variable(inputs)
        with torch.enable_grad():
            outputs = ctx.run_function(*detached_inputs)
        torch.set_rng_state(bwd_cpu_rng_state)
        _set_device_rng_state(bwd_cuda_rng_state)
        get_cuda_rng_tracker().set_states(bwd_cuda_rng_state_tracker)
        _COUNTER_RNG_STREAMS.set_states(bwd_counter_streams)
        if isinstance(outputs, torch.Tensor):
            outputs = (outputs,)
        torch.autograd.backward(outputs, args)
        grads = tuple(inp.grad if isinstance(inp, torch.Tensor) else inp for inp in detached_inputs)
        return (None, None) + grads


def checkpoint(function, *args, distribute_saved_activations=None):
    """Checkpoint ``function(*args)``.  The first input is stored 1/tp-split across the TP group
    when ``distribute_saved_activations`` (default: when the activation buffer was initialised)."""
    if distribute_saved_activations is None:
        distribute_saved_activations = _CHECKPOINTED_ACTIVATIONS_MEMORY_BUFFER is not None
    return CheckpointFunction.apply(function, distribute_saved_activations, *args)
