"""Arena buffers for checkpointed activations (reference
apex/transformer/tensor_parallel/memory.py:22-136).

With 288 GB of HBM per MI355X the point is fragmentation control, not capacity: each purpose
gets ONE contiguous device tensor that tensors are bump-allocated from (``add`` copies into the
next free slice and returns that view) and that is recycled as a whole every iteration
(``reset``).  A ring of arenas lets consecutive micro-batches keep their checkpoints alive until
their backward.  Public API as in the reference: ``allocate_mem_buff``, ``get_mem_buff``,
``MemoryBuffer`` and ``RingMemBuffer``."""
import torch

_ARENAS = {}


def _rank0():
    d = torch.distributed
    return not d.is_initialized() or d.get_rank() == 0


def _device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def allocate_mem_buff(name, numel, dtype, track_usage):
    """Create and register the arena ``name`` (names are unique)."""
    if name in _ARENAS:
        raise RuntimeError("memory buffer {!r} is already allocated".format(name))
    buf = _ARENAS[name] = MemoryBuffer(name, numel, dtype, track_usage)
    return buf


def get_mem_buff(name):
    return _ARENAS[name]


class MemoryBuffer:
    """Bump allocator over one contiguous ``numel``-element tensor of ``dtype``."""

    def __init__(self, name, numel, dtype, track_usage, device=None):
        self.name, self.numel, self.dtype = name, int(numel), dtype
        self.data = torch.empty(self.numel, dtype=dtype, device=device or _device())
        self._used = 0
        self.track_usage = track_usage
        self._usage = [0.0, 0.0]  # (elements handed out, capacity) summed over get_data() calls
        if _rank0():
            mb = self.numel * self.data.element_size() / 2 ** 20
            print("> building the {} memory buffer with {} num elements and {} dtype ({:.1f} MB)...".format(
                name, self.numel, dtype, mb), flush=True)

    # the reference exposes these two as attributes
    @property
    def in_use_value(self):
        return self._usage[0]

    @property
    def total_value(self):
        return self._usage[1]

    def reset(self):
        self._used = 0

    def is_in_use(self):
        return self._used > 0

    def numel_in_use(self):
        return self._used

    def add(self, tensor):
        """Copy ``tensor`` into the next free slice; returns the view shaped like ``tensor``."""
        if tensor.dtype != self.dtype:
            raise TypeError("tensor dtype {} does not match buffer dtype {}".format(tensor.dtype, self.dtype))
        n = tensor.numel()
        if self._used + n > self.numel:
            raise RuntimeError("memory buffer {!r} exhausted: need {} more elements, {} free".format(
                self.name, n, self.numel - self._used))
        view = self.data.narrow(0, self._used, n).view(tensor.shape)
        self._used += n
        view.copy_(tensor)
        return view

    def get_data(self):
        """The allocated prefix of the arena."""
        if self.track_usage:
            self._usage[0] += self._used
            self._usage[1] += self.numel
        return self.data.narrow(0, 0, self._used)

    def print_average_usage(self):
        if not self.track_usage:
            raise RuntimeError("usage tracking is disabled for memory buffer {!r}".format(self.name))
        if _rank0():
            print(" > usage of {} memory buffer: {:.2f} %".format(
                self.name, 100.0 * self._usage[0] / max(self._usage[1], 1.0)), flush=True)


class RingMemBuffer:
    """``num_buffers`` arenas used round-robin; taking one that still holds data is an error."""

    def __init__(self, name, num_buffers, numel, dtype, track_usage):
        self.num_buffers = num_buffers
        self.buffers = [allocate_mem_buff("{} {}".format(name, i), numel, dtype, track_usage)
                        for i in range(num_buffers)]
        self._next = 0

    def get_next_buffer(self):
        buf = self.buffers[self._next]
        self._next = (self._next + 1) % self.num_buffers
        if buf.is_in_use():
            raise RuntimeError("memory buffer {!r} is still in use".format(buf.name))
        return buf
