"""Shared plumbing of the legacy contrib optimizers (``fused_adam``, ``fused_sgd``, ``fused_lamb``:
reference apex/contrib/optimizers/fused_adam.py:6-206, fused_sgd.py:7-211, fused_lamb.py:6-208),
which ``apex.contrib.optimizers.FP16_Optimizer`` drives.

Their ``step`` receives the (loss-scaled, possibly fp16) gradients, the fp32 master params are
``group['params']`` and an optional reduced-precision copy is written out.  Each group is one
multi-tensor launch per dtype combination on the gfx950 engine (``amp_C``); the loss scale and
max-grad-norm clip are folded into a single device inverse-scale factor consumed by the kernel.
"""
import types


def _groupify(x, n):
    if x is None:
        return [None] * n
    if isinstance(x, types.GeneratorType):
        return [list(x)]
    x = list(x)
    if x and not isinstance(x[0], (list, tuple)):
        return [x]
    return x


def _split_by(keys, *lists):
    """Partition parallel lists by a key (dtype tuple) so each multi-tensor launch is homogeneous."""
    out = {}
    for i, k in enumerate(keys):
        slot = out.setdefault(k, [[] for _ in lists])
        for j, lst in enumerate(lists):
            slot[j].append(lst[i])
    return out
