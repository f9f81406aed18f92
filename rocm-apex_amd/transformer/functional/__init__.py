from .fused_softmax import FusedScaleMaskSoftmax  # noqa: F401
from .fused_softmax import scaled_masked_softmax, scaled_upper_triang_masked_softmax, scaled_softmax  # noqa: F401

__all__ = ["FusedScaleMaskSoftmax"]
