from .grad_scaler import GradScaler  # noqa: F401

__all__ = ["GradScaler"]
