from .schedules import get_forward_backward_func  # noqa: F401
from .schedules.common import build_model  # noqa: F401

__all__ = ["get_forward_backward_func", "build_model"]
