"""Contiguous activation buffers for checkpointed activations
(reference apex/transformer/tensor_parallel/memory.py:22-136).

With 288 GB of HBM per MI355X the point of these buffers is fragmentation control, not
capacity: one large arena per purpose, bump-allocated and reset every iteration."""
import torch

_MEM_BUFFS = dict()


def allocate_mem_buff(name, numel, dtype, track_usage):
    assert name not in _MEM_BUFFS, "memory buffer {} already allocated.".format(name)
    _MEM_BUFFS[name] = MemoryBuffer(name, numel, dtype, track_usage)
    return _MEM_BUFFS[name]


def get_mem_buff(name):
    return _MEM_BUFFS[name]


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class MemoryBuffer:
    """A bump allocator over one contiguous tensor: ``add(t)`` copies ``t`` into the next free
    slice and returns that view; ``reset()`` recycles the whole arena."""

    def __init__(self, name, numel, dtype, track_usage, device=None):
        if not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0:
            element_size = torch.tensor([], dtype=dtype).element_size()
            print("> building the {} memory buffer with {} num elements and {} dtype ({:.1f} MB)...".format(
                name, numel, dtype, numel * element_size / 1024 / 1024), flush=True)
        self.name = name
        self.numel = numel
        self.dtype = dtype
        self.data = torch.empty(self.numel, dtype=self.dtype, device=device or _default_device(), requires_grad=False)
        self._start = 0
        self.track_usage = track_usage
        if self.track_usage:
            self.in_use_value = 0.0
            self.total_value = 0.0

    def reset(self):
        self._start = 0

    def is_in_use(self):
        return self._start > 0

    def numel_in_use(self):
        return self._start

    def add(self, tensor):
        assert tensor.dtype == self.dtype, "Input tensor type {} different from buffer type {}".format(
            tensor.dtype, self.dtype)
        tensor_numel = torch.numel(tensor)
        new_start = self._start + tensor_numel
        assert new_start <= self.numel, "Not enough memory left in the buffer ({} > {})".format(
            tensor_numel, self.numel - self._start)
        new_tensor = self.data[self._start:new_start]
        self._start = new_start
        new_tensor = new_tensor.view(tensor.shape)
        new_tensor.copy_(tensor)
        return new_tensor

    def get_data(self):
        if self.track_usage:
            self.in_use_value += float(self._start)
            self.total_value += float(self.numel)
        return self.data[:self._start]

    def print_average_usage(self):
        assert self.track_usage, "You need to enable track usage."
        if not torch.distributed.is_initialized() or torch.distributed.get_rank() == 0:
            print(" > usage of {} memory buffer: {:.2f} %".format(
                self.name, self.in_use_value * 100.0 / self.total_value), flush=True)


class RingMemBuffer:
    """A ring of memory buffers."""

    def __init__(self, name, num_buffers, numel, dtype, track_usage):
        self.num_buffers = num_buffers
        self.buffers = [allocate_mem_buff(name + " {}".format(i), numel, dtype, track_usage)
                        for i in range(num_buffers)]
        self._index = -1

    def get_next_buffer(self):
        self._index = (self._index + 1) % self.num_buffers
        buff = self.buffers[self._index]
        assert not buff.is_in_use(), "buffer is already in use."
        return buff
