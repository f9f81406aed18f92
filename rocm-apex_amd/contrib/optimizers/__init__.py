"""Contrib optimizers (reference apex/contrib/optimizers/__init__.py)."""
from .distributed_fused_adam import DistributedFusedAdam  # noqa: F401
from .distributed_fused_adam_v2 import DistributedFusedAdamV2  # noqa: F401
from .distributed_fused_adam_v3 import DistributedFusedAdamV3  # noqa: F401
from .distributed_fused_lamb import DistributedFusedLAMB  # noqa: F401
from .fp16_optimizer import FP16_Optimizer  # noqa: F401
from .fused_adam import FusedAdam  # noqa: F401
from .fused_lamb import FusedLAMB  # noqa: F401
from .fused_sgd import FusedSGD  # noqa: F401
