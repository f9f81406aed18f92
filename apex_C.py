"""Top-level ``apex_C`` module name kept for callers written against the reference
(``import apex_C; flat = apex_C.flatten(grads)``)."""
from apex.apex_C import flatten, unflatten  # noqa: F401
