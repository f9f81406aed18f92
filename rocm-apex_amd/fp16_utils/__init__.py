"""Legacy fp16 helpers (reference apex/fp16_utils/__init__.py)."""
from .fp16util import (BN_convert_float, network_to_half, prep_param_lists,  # noqa: F401
                       model_grads_to_master_grads, master_params_to_model_params, tofp16, to_python_float,
                       clip_grad_norm, convert_module, convert_network, FP16Model)
from .fp16_optimizer import FP16_Optimizer  # noqa: F401
from .loss_scaler import LossScaler, DynamicLossScaler  # noqa: F401
