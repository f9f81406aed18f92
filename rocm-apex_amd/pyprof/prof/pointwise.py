"""Elementwise ops (reference apex/pyprof/prof/pointwise.py, activation.py, dropout.py,
convert.py, misc.py): unary / binary / ternary math with broadcasting, activations, dropout,
dtype conversions.  Output numel = broadcast of the tensor operands; bytes = every tensor
operand read once + the output written once (in-place ops write into their first operand).
FLOPs per output element come from ``COST`` (transcendentals are priced as a few FLOPs, as in
the reference)."""
from .base import OpModel
from .utility import broadcast, fmt_shape, nbytes_of, numel, short

COST = {
    # arithmetic
    "add": 1, "sub": 1, "mul": 1, "div": 1, "true_divide": 1, "floor_divide": 1, "remainder": 2, "fmod": 2,
    "rsub": 1, "neg": 1, "abs": 1, "reciprocal": 1, "sign": 1, "square": 1, "pow": 2, "float_power": 2,
    "addcmul": 2, "addcdiv": 2, "lerp": 3, "clamp": 2, "clip": 2, "clamp_min": 1, "clamp_max": 1,
    "maximum": 1, "minimum": 1, "fmax": 1, "fmin": 1, "hypot": 4, "atan2": 8, "ceil": 1, "floor": 1,
    "round": 1, "trunc": 1, "frac": 2,
    # transcendental
    "exp": 4, "exp2": 4, "expm1": 4, "log": 4, "log2": 4, "log10": 4, "log1p": 4, "sqrt": 2, "rsqrt": 2,
    "sin": 4, "cos": 4, "tan": 6, "asin": 8, "acos": 8, "atan": 8, "sinh": 6, "cosh": 6, "tanh": 5,
    "sigmoid": 4, "erf": 6, "erfc": 6, "erfinv": 10, "logit": 5, "xlogy": 5,
    # comparisons / logic
    "eq": 1, "ne": 1, "lt": 1, "le": 1, "gt": 1, "ge": 1, "logical_and": 1, "logical_or": 1, "logical_not": 1,
    "logical_xor": 1, "bitwise_and": 1, "bitwise_or": 1, "bitwise_xor": 1, "bitwise_not": 1, "isnan": 1,
    "isinf": 1, "isfinite": 1, "where": 1, "nan_to_num": 2,
    # activations
    "relu": 1, "relu6": 2, "leaky_relu": 2, "elu": 5, "selu": 6, "celu": 6, "gelu": 9, "silu": 5, "mish": 12,
    "hardtanh": 2, "hardsigmoid": 3, "hardswish": 4, "hardshrink": 2, "softshrink": 3, "tanhshrink": 6,
    "softplus": 8, "softsign": 3, "threshold": 1, "prelu": 2, "rrelu": 3, "glu": 5, "logsigmoid": 8,
    # dropout (mask generation + scale)
    "dropout": 3, "alpha_dropout": 4, "feature_alpha_dropout": 4, "dropout1d": 3, "dropout2d": 3,
    "dropout3d": 3, "feature_dropout": 3,
}
ALIASES = {"__add__": "add", "__radd__": "add", "__iadd__": "add", "__sub__": "sub", "__rsub__": "rsub",
           "__isub__": "sub", "__mul__": "mul", "__rmul__": "mul", "__imul__": "mul", "__truediv__": "div",
           "__rtruediv__": "div", "__itruediv__": "div", "__div__": "div", "__floordiv__": "floor_divide",
           "__mod__": "remainder", "__pow__": "pow", "__rpow__": "pow", "__neg__": "neg", "__abs__": "abs",
           "__eq__": "eq", "__ne__": "ne", "__lt__": "lt", "__le__": "le", "__gt__": "gt", "__ge__": "ge",
           "__and__": "bitwise_and", "__or__": "bitwise_or", "__xor__": "bitwise_xor", "__invert__": "bitwise_not",
           "__iand__": "bitwise_and", "__ior__": "bitwise_or", "__ixor__": "bitwise_xor", "multiply": "mul",
           "divide": "div", "subtract": "sub", "greater": "gt", "less": "lt", "absolute": "abs", "negative": "neg"}


def canonical(op):
    op = ALIASES.get(op, op)
    if op.endswith("_") and not op.startswith("__"):
        op = op[:-1]
    return ALIASES.get(op, op)


class Pointwise(OpModel):
    kind = "pointwise"

    def parse(self):
        self.name = canonical(self.rec.get("op", ""))
        if self.rec.get("op") == "forward":
            mod = self.rec.get("mod", "")
            self.name = {"LeakyReLU": "leaky_relu", "AlphaDropout": "alpha_dropout"}.get(mod, mod.lower())
        self.inplace = self.rec.get("op", "").endswith("_") and not self.rec.get("op", "").startswith("__") or \
            self.rec.get("op", "").startswith("__i")
        shapes = [t["shape"] for t in self.ts]
        self.out = broadcast(*shapes) if shapes else ()
        self.dtype = self.ts[0].get("dtype", "float32") if self.ts else "float32"
        if self.name in ("eq", "ne", "lt", "le", "gt", "ge", "isnan", "isinf", "isfinite") or \
                self.name.startswith("logical_"):
            self.out_dtype = "bool"
        else:
            self.out_dtype = self.dtype

    def fwd_flops(self):
        return COST.get(self.name, 1) * numel(self.out)

    def fwd_bytes(self):
        rd = sum(numel(t["shape"]) * nbytes_of(t.get("dtype")) for t in self.ts)
        return rd + numel(self.out) * nbytes_of(self.out_dtype)

    def bprop_flops(self):  # grad of y=f(x): one multiply by f'(x) (f' itself ~ the forward cost)
        return (COST.get(self.name, 1) + 1) * numel(self.out)

    def bprop_bytes(self):
        return self.fwd_bytes() + numel(self.out) * nbytes_of(self.dtype)

    def params(self):
        return {"T": fmt_shape(self.out), "type": short(self.dtype)}


class Convert(OpModel):
    """``to`` / ``type`` / ``float`` / ``half`` / ``bfloat16`` / ``copy_``: read + write."""
    kind = "convert"

    def parse(self):
        op = self.rec.get("op", "")
        self.src = self.ts[0].get("dtype", "float32") if self.ts else "float32"
        dst = {"float": "float32", "half": "float16", "bfloat16": "bfloat16", "double": "float64", "int": "int32",
               "long": "int64", "bool": "bool", "byte": "uint8", "char": "int8"}.get(op)
        if dst is None:
            for a in self.args:
                if a.get("type") == "dtype":
                    dst = a.get("value")
            if op == "copy_" and len(self.ts) > 1:
                dst, self.src = self.ts[0].get("dtype"), self.ts[1].get("dtype")
        self.dst = dst or self.src
        self.n = numel(self.ts[0]["shape"]) if self.ts else 0

    def fwd_flops(self):
        return 0

    def fwd_bytes(self):
        if self.src == self.dst and self.rec.get("op") in ("to", "type", "float", "half", "bfloat16"):
            return 0  # no-op conversion returns self
        return self.n * (nbytes_of(self.src) + nbytes_of(self.dst))

    def params(self):
        return {"T": self.n, "src": short(self.src), "dst": short(self.dst)}


OPS = {}
for _op in list(COST) + list(ALIASES):
    OPS[_op] = Pointwise
    if not _op.startswith("__"):
        OPS[_op + "_"] = Pointwise
for _op in ("to", "type", "float", "half", "bfloat16", "double", "int", "long", "bool", "byte", "char", "copy_",
            "type_as"):
    OPS[_op] = Convert
MODULES = {m: Pointwise for m in ("ReLU", "ReLU6", "LeakyReLU", "ELU", "SELU", "CELU", "GELU", "SiLU", "Mish",
                                  "Hardtanh", "Hardsigmoid", "Hardswish", "Hardshrink", "Softshrink", "Tanhshrink",
                                  "Softplus", "Softsign", "Threshold", "PReLU", "RReLU", "GLU", "LogSigmoid",
                                  "Sigmoid", "Tanh", "Dropout", "Dropout1d", "Dropout2d", "Dropout3d", "AlphaDropout")}
