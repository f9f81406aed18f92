"""``multi_tensor_applier`` (reference apex/multi_tensor_apply/__init__.py:3)."""
from .multi_tensor_apply import MultiTensorApply

# 64K-element chunks, as in the reference; on gfx950 one chunk is 32 steps of a 256-lane block
# moving 8 elements per lane.
multi_tensor_applier = MultiTensorApply(2048 * 32)
