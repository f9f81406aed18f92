"""Megatron-style model parallelism for MI355X (reference apex/transformer/__init__.py).

Submodules: ``parallel_state`` (TP/PP/DP process groups over RCCL), ``tensor_parallel``
(column/row/vocab-parallel layers, mappings, vocab-parallel cross entropy, RNG tracker,
activation checkpointing), ``pipeline_parallel`` (p2p + no-pipelining / 1F1B / interleaved
schedules), ``functional`` (fused scale-mask-softmax), ``amp`` (model-parallel GradScaler)."""
import importlib

from .enums import AttnMaskType, AttnType, LayerType  # noqa: F401
from . import functional  # noqa: F401

_LAZY = ("amp", "parallel_state", "pipeline_parallel", "tensor_parallel", "utils", "microbatches", "log_util",
         "testing", "layers", "_data")

__all__ = ["amp", "functional", "parallel_state", "pipeline_parallel", "tensor_parallel", "utils",
           "LayerType", "AttnType", "AttnMaskType"]


def __getattr__(name):
    if name in _LAZY:
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
