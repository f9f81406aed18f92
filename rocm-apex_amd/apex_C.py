"""``apex_C``: flatten / unflatten of dense tensor lists (reference csrc/flatten_unflatten.cpp:4-18).

The DDP in this framework reduces gradients out of persistent flat buckets (no per-step
flatten), so these are only the compatibility entry points; both are single fused torch ops
(one cat / zero-copy views)."""
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


def flatten(tensors):
    return _flatten_dense_tensors(list(tensors))


def unflatten(flat, tensors):
    return list(_unflatten_dense_tensors(flat, list(tensors)))
