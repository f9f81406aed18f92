"""Automatic mixed precision (reference apex/amp/__init__.py:1-4)."""
from .amp import (init, half_function, bfloat16_function, float_function, promote_function,  # noqa: F401
                  register_half_function, register_bfloat16_function, register_float_function,
                  register_promote_function)
from .handle import scale_loss, disable_casts  # noqa: F401
from .frontend import initialize, state_dict, load_state_dict  # noqa: F401
from ._amp_state import master_params, _amp_state  # noqa: F401
