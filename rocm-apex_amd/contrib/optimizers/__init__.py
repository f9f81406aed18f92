"""Contrib optimizers (reference apex/contrib/optimizers/__init__.py)."""
from .distributed_fused_adam import (DistributedFusedAdam, DistributedFusedAdamV2,  # noqa: F401
                                     DistributedFusedAdamV3)
from .distributed_fused_lamb import DistributedFusedLAMB  # noqa: F401
from .fp16_optimizer import FP16_Optimizer  # noqa: F401
from .fused_legacy import FusedAdam, FusedLAMB, FusedSGD  # noqa: F401
