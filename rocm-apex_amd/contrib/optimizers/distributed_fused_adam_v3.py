"""DistributedFusedAdamV3: all-reduce + sharded step + all-gather (reference
apex/contrib/optimizers/distributed_fused_adam_v3.py:7-325)."""
from .distributed_fused_adam import DistributedFusedAdam


class DistributedFusedAdamV3(DistributedFusedAdam):
    """Reference v3 (apex/contrib/optimizers/distributed_fused_adam_v3.py:7-325): every block is
    ALL-REDUCED whole, the sharded fused step runs on this rank's slice of the result and the
    parameters are all-gathered.  Moves twice the reduce bytes of the reduce-scatter
    variant; results are identical."""

    def __init__(self, *args, **kwargs):
        kwargs["_reduction_mode"] = "ar"
        super().__init__(*args, **kwargs)
