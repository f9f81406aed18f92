"""Fused ResNet bottleneck blocks (reference apex/contrib/bottleneck/__init__.py)."""
from .bottleneck import Bottleneck, FrozenBatchNorm2d, SpatialBottleneck  # noqa: F401
from .halo_exchangers import halo_pad  # noqa: F401
