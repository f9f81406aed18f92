"""Graph-safe dropout randomness for the native dropout kernels (flash attention, fused
bias-dropout-add).

Those kernels regenerate their keep masks from a counter-based hash of (seed, offset); seed and
offset come from the host (the model's seed and the Megatron counter streams,
``tensor_parallel.get_counter_rng_streams``).  Inside a captured hipGraph the host values are
frozen at capture time, so every replay would redraw the SAME masks.  With device RNG steps
enabled, each launch additionally gets a pointer to a per-device int64 step counter and uses
``offset + (step << 32)``; ``advance()`` bumps that counter ON THE DEVICE (one tiny kernel, itself
capturable), so a graph that starts with ``advance()`` draws fresh masks on every replay while the
forward and the backward of one call always agree: each forward launches with a snapshot of the
counter (``snapshot()``) and saves that snapshot for its backward.

Eager code that never calls ``enable()`` is unaffected (no pointer is passed)."""
import os

import torch

_ENABLED = [False]
_STEPS = {}
# device -> the snapshot shared by every dropout call since the last advance(): the counter only
# changes in advance(), so one copy per step serves them all (a GPT-2 medium step has 72 dropout
# calls; a copy each was 72 x 4.8 us of D2D copy launches per step)
_SNAPS = {}
_SHARE = os.environ.get("APEX_AMD_RNG_SHARED_SNAPSHOT", "1") != "0"  # A/B knob


def enable(flag=True):
    _ENABLED[0] = bool(flag)
    _SNAPS.clear()


def enabled():
    return _ENABLED[0]


def step_tensor(device):
    """The device's int64[1] step counter when device steps are enabled (else None)."""
    if not _ENABLED[0]:
        return None
    device = torch.device(device)
    if device.type != "cuda":
        return None
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = _STEPS.get(key)
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=torch.device("cuda", key))
        _STEPS[key] = t
    return t


def snapshot(device):
    """A private copy of the step counter for ONE dropout call (None when device steps are off).

    The forward launches with the copy and saves it for the backward, so the backward rebuilds
    exactly the forward's mask even when ``advance()`` runs in between (gradient accumulation,
    pipeline 1F1B with several forwards in flight, recompute).  A D2D copy (capturable), made once
    after each ``advance()`` and shared by the calls until the next one (a snapshot is never
    written after it is taken)."""
    t = step_tensor(device)
    if t is None:
        return None
    if not _SHARE:
        return t.clone()
    # a snapshot is only shared within one capture state: one taken eagerly (e.g. warm-up with no
    # trailing advance()) must not be reused inside a graph capture, whose replays would then all
    # read that frozen copy instead of a clone made by the graph itself — and vice versa
    capturing = torch.cuda.is_current_stream_capturing()
    hit = _SNAPS.get(t.device.index)
    if hit is None or hit[0] != capturing:
        hit = (capturing, t.clone())
        _SNAPS[t.device.index] = hit
    return hit[1]


def advance(device=None):
    """Next step's masks: increments the device counter in stream order (capturable)."""
    t = step_tensor(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
    if t is not None:
        t.add_(1)
        _SNAPS.pop(t.device.index, None)


def effective_offset(offset, device):
    """Host-side equivalent of the kernels' offset (reference / CPU paths; reads the counter)."""
    t = step_tensor(device)
    return int(offset) + ((int(t.item()) << 32) if t is not None else 0)
