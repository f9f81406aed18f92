"""Packed variable-length fused attention (reference apex/contrib/fmha/__init__.py)."""
from .fmha import FMHA, FMHAFun  # noqa: F401
