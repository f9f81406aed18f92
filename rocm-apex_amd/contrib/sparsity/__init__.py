"""Automatic structured sparsity (reference apex/contrib/sparsity/__init__.py)."""
from .asp import ASP  # noqa: F401
from .sparse_masklib import create_mask  # noqa: F401
