"""Top-level ``amp_C`` module name kept for callers written against the reference
(``import amp_C; multi_tensor_applier(amp_C.multi_tensor_adam, ...)``)."""
from apex.amp_C import *  # noqa: F401,F403
from apex.amp_C import __all__  # noqa: F401
