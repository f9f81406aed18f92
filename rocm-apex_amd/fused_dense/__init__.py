from .fused_dense import (FusedDense, FusedDenseGeluDense, DenseNoBiasFunc, FusedDenseFunc,  # noqa: F401
                          FusedDenseGeluDenseFunc, fused_dense_function, dense_no_bias_function,
                          fused_dense_gelu_dense_function)
from .fused_dense import maybe_sync_lt_plans, sync_lt_plans  # noqa: F401,E402
