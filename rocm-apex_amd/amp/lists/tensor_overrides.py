"""O1/O4 cast policy for ``torch.Tensor`` methods (reference apex/amp/lists/tensor_overrides.py).
Every torch-namespace entry that is also a Tensor method is included."""
import torch

from . import torch_overrides

MODULE = torch.Tensor

FP16_FUNCS = ["__matmul__"]
BFLOAT16_FUNCS = ["__matmul__"]
FP32_FUNCS = ["__ipow__", "__pow__", "__rpow__", "cpu"]
CASTS = ["__add__", "__div__", "__eq__", "__ge__", "__gt__", "__iadd__", "__idiv__", "__imul__", "__isub__",
         "__itruediv__", "__le__", "__lt__", "__mul__", "__ne__", "__radd__", "__rdiv__", "__rmul__", "__rsub__",
         "__rtruediv__", "__sub__", "__truediv__"]
SEQUENCE_CASTS = []

for _name in ("FP16_FUNCS", "BFLOAT16_FUNCS", "FP32_FUNCS", "CASTS", "SEQUENCE_CASTS"):
    _lst = globals()[_name]
    for _fn in getattr(torch_overrides, _name):
        if hasattr(MODULE, _fn) and _fn not in _lst:
            _lst.append(_fn)
    globals()[_name] = [f for f in _lst if hasattr(MODULE, f)]
