"""Fused optimizers (reference apex/optimizers/__init__.py)."""
from .fused_sgd import FusedSGD  # noqa: F401
from .fused_adam import FusedAdam  # noqa: F401
from .fused_novograd import FusedNovoGrad  # noqa: F401
from .fused_lamb import FusedLAMB  # noqa: F401
from .fused_adagrad import FusedAdagrad  # noqa: F401
from .fused_mixed_precision_lamb import FusedMixedPrecisionLamb  # noqa: F401
