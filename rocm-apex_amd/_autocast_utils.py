"""Autocast helpers for fused autograd Functions (reference apex/_autocast_utils.py:6-17)."""
from typing import Optional, Sequence

import torch


def _get_autocast_dtypes() -> Sequence[torch.dtype]:
    return [torch.half, torch.bfloat16]


def _get_current_dtype(dtype: Optional[torch.dtype] = None) -> torch.dtype:
    if not torch.is_autocast_enabled():
        return torch.float or dtype
    return torch.get_autocast_gpu_dtype()


def _cast_if_autocast_enabled(*args):
    if not torch.is_autocast_enabled():
        return args
    return torch.cuda.amp.autocast_mode._cast(args, torch.get_autocast_gpu_dtype())
