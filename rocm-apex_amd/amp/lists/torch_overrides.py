"""O1/O4 cast policy for the ``torch`` namespace (reference apex/amp/lists/torch_overrides.py).
On ROCm the batched GEMMs are always safe in reduced precision (rocBLAS/hipBLASLt)."""
import torch

MODULE = torch

FP16_FUNCS = ["conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d", "conv_transpose3d",
              "conv_tbc", "prelu", "addmm", "addmv", "addr", "matmul", "mm", "mv",
              "addbmm", "baddbmm", "bmm"]
BFLOAT16_FUNCS = ["conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d", "conv_transpose3d",
                  "conv_tbc", "addmm", "addmv", "addr", "matmul", "mm", "mv",
                  "addbmm", "baddbmm", "bmm"]

FP32_FUNCS = ["acos", "asin", "cosh", "erfinv", "exp", "expm1", "log", "log10", "log2", "reciprocal", "rsqrt",
              "sinh", "tan", "pow", "cumprod", "cumsum", "dist", "norm", "prod", "std", "sum", "var", "renorm"]

CASTS = ["addcdiv", "addcmul", "atan2", "cross", "bilinear", "dot", "add", "div", "mul",
         "eq", "equal", "ge", "gt", "le", "lt", "ne"]

SEQUENCE_CASTS = ["cat", "stack"]
