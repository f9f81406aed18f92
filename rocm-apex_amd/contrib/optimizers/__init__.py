"""Contrib optimizers (reference apex/contrib/optimizers/__init__.py)."""
from .fp16_optimizer import FP16_Optimizer  # noqa: F401
