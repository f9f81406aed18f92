"""Autocast helpers for fused autograd Functions (reference apex/_autocast_utils.py:6-17).

The fused Functions run their own mixed-precision kernels, so at the Function boundary the
floating-point arguments are cast ONCE to the active autocast dtype and autocast is switched
off inside (otherwise forward would run autocast-cast GEMMs while backward sees the uncast
saved tensors).  Both device autocasts are honoured: "cuda" (HIP on ROCm) and "cpu" — the CPU
tier runs the same Functions under ``torch.autocast("cpu", dtype=torch.bfloat16)``."""
import contextlib
from typing import Optional, Sequence

import torch

_DEVICES = ("cuda", "cpu")


def _get_autocast_dtypes() -> Sequence[torch.dtype]:
    return [torch.half, torch.bfloat16]


def _active_device() -> Optional[str]:
    for dev in _DEVICES:
        if torch.is_autocast_enabled(dev):
            return dev
    return None


def _get_current_dtype(dtype: Optional[torch.dtype] = None) -> torch.dtype:
    dev = _active_device()
    if dev is None:
        return dtype or torch.float
    return torch.get_autocast_dtype(dev)


def _cast_if_autocast_enabled(*args):
    dev = _active_device()
    if dev is None:
        return args
    return torch.amp.autocast_mode._cast(args, dev, torch.get_autocast_dtype(dev))


@contextlib.contextmanager
def _autocast_disabled():
    """Autocast off for every device type inside a fused Function call."""
    with torch.autocast("cuda", enabled=False), torch.autocast("cpu", enabled=False):
        yield
