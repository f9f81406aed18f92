"""Device-time accounting of the collectives that sit on a training step's critical path, so a
multi-GPU benchmark line explains itself (bench.py reports ``allreduce_exposed_ms`` and
``bn_exchange_ms_per_step``).

Spans are pairs of events recorded on the CURRENT stream around the host code that issues a
collective and waits for it: the elapsed time between them is the time the compute stream was
held by that collective (for DDP: from the end of backward to the last gradient bucket's
completion — the all-reduce time NOT hidden under backward; for a synchronized batch norm: the
statistics / backward-sum exchange).  Off by default (event records cost host time per call);
``enable()`` for a few measurement steps, then ``summary()`` (which synchronizes)."""
import contextlib
import time

import torch

_ENABLED = False
_SPANS = {}


def enable(flag=True):
    global _ENABLED
    _ENABLED = bool(flag)


def enabled():
    return _ENABLED


def reset():
    _SPANS.clear()


@contextlib.contextmanager
def span(name, device=None):
    """Record the device time of the enclosed collective issue + wait under ``name``."""
    if not _ENABLED:
        yield
        return
    use_events = torch.cuda.is_available() and (device is None or getattr(device, "type", "cuda") == "cuda")
    if use_events:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            yield
        finally:
            e.record()
            _SPANS.setdefault(name, []).append((s, e))
    else:
        t0 = time.perf_counter()
        try:
            yield
        finally:
            _SPANS.setdefault(name, []).append((t0, time.perf_counter()))


def total_ms(name):
    """Sum of the recorded spans of ``name`` in milliseconds (synchronizes the device)."""
    rows = _SPANS.get(name, [])
    if not rows:
        return 0.0
    if isinstance(rows[0][0], float):
        return sum((b - a) * 1000.0 for a, b in rows)
    torch.cuda.synchronize()
    return sum(float(a.elapsed_time(b)) for a, b in rows)


def count(name):
    return len(_SPANS.get(name, []))


def summary(steps):
    """{name: ms per step} over ``steps`` measured steps."""
    steps = max(1, int(steps))
    return {name: round(total_ms(name) / steps, 4) for name in sorted(_SPANS)}
