"""Named interval timers for the pipeline schedules (reference
apex/transformer/pipeline_parallel/_timers.py:6-83, which brackets every start / stop with a
full ``torch.cuda.synchronize()`` and reads the host clock).

Here an interval is a pair of HIP events recorded on the current stream: ``start()`` / ``stop()``
never block the host or the device, so timing a pipeline stage does not serialize its RCCL
overlap.  The device is waited on lazily, only for the last stop event, when a value is read
(``elapsed`` / ``log`` / ``write``).  Without a GPU the host monotonic clock is used.  Public
surface kept: ``_Timers()(name).start() / .stop() / .reset() / .elapsed(reset)``,
``_Timers.log(names, normalizer, reset)`` and ``_Timers.write(names, writer, iteration, ...)``."""
import time

import torch


class _Interval:
    __slots__ = ("begin", "end")

    def __init__(self, begin, end=None):
        self.begin, self.end = begin, end


class _Timer:
    def __init__(self, name):
        self.name_ = name
        self._gpu = torch.cuda.is_available()
        self._closed = []     # finished intervals not yet folded into _seconds
        self._open = None     # running interval
        self._seconds = 0.0

    @property
    def started_(self):
        return self._open is not None

    def _mark(self):
        if self._gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def start(self):
        if self._open is not None:
            raise RuntimeError("timer {!r} has already been started".format(self.name_))
        self._open = _Interval(self._mark())

    def stop(self):
        if self._open is None:
            raise RuntimeError("timer {!r} is not started".format(self.name_))
        self._open.end = self._mark()
        self._closed.append(self._open)
        self._open = None

    def _fold(self):
        if not self._closed:
            return
        if self._gpu:
            self._closed[-1].end.synchronize()  # events complete in stream order
            self._seconds += sum(iv.begin.elapsed_time(iv.end) for iv in self._closed) / 1000.0
        else:
            self._seconds += sum(iv.end - iv.begin for iv in self._closed)
        self._closed = []

    def reset(self):
        self._closed = []
        self._open = None
        self._seconds = 0.0

    def elapsed(self, reset=True):
        """Seconds accumulated so far (a running interval counts up to now and keeps running)."""
        running = self._open is not None
        if running:
            self.stop()
        self._fold()
        total = self._seconds
        if reset:
            self.reset()
        if running:
            self.start()
        return total


class _Timers:
    """``timers(name)`` creates or returns a named timer."""

    def __init__(self):
        self.timers = {}

    def __call__(self, name):
        t = self.timers.get(name)
        if t is None:
            t = self.timers[name] = _Timer(name)
        return t

    def _values_ms(self, names, normalizer, reset):
        if normalizer <= 0.0:
            raise ValueError("normalizer must be positive")
        return [(n, self.timers[n].elapsed(reset=reset) * 1000.0 / normalizer) for n in names]

    def write(self, names, writer, iteration, normalizer=1.0, reset=False):
        """Scalars ``<name>-time`` (seconds) to a TensorBoard-style ``writer``."""
        for name, ms in self._values_ms(names, normalizer, reset):
            writer.add_scalar(name + "-time", ms / 1000.0, iteration)

    def log(self, names, normalizer=1.0, reset=True):
        """One ``time (ms) | name: value ...`` line, printed by the last rank (the pipeline's last
        stage) or by the only process."""
        line = "time (ms)" + "".join(" | {}: {:.2f}".format(n, ms) for n, ms in
                                     self._values_ms(names, normalizer, reset))
        dist = torch.distributed
        if not dist.is_initialized() or dist.get_rank() == dist.get_world_size() - 1:
            print(line, flush=True)
