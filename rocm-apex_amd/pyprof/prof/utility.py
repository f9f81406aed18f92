"""Helpers shared by the op models (reference apex/pyprof/prof/utility.py): dtype sizes,
argument lookup in marker descriptions, broadcasting."""
import math

DTYPE_BYTES = {
    "float64": 8, "double": 8, "float32": 4, "float": 4, "float16": 2, "half": 2, "bfloat16": 2,
    "float8_e4m3fn": 1, "float8_e5m2": 1, "float8_e4m3fnuz": 1, "float8_e5m2fnuz": 1,
    "int64": 8, "long": 8, "int32": 4, "int": 4, "int16": 2, "int8": 1, "uint8": 1, "bool": 1,
    "complex64": 8, "complex128": 16,
}
SHORT = {"float32": "fp32", "float16": "fp16", "bfloat16": "bf16", "float64": "fp64", "int64": "i64",
         "int32": "i32", "uint8": "u8", "int8": "i8", "bool": "b", "float8_e4m3fn": "fp8e4m3",
         "float8_e5m2": "fp8e5m2"}


def nbytes_of(dtype):
    return DTYPE_BYTES.get(str(dtype), 4)


def short(dtype):
    return SHORT.get(str(dtype), str(dtype))


def numel(shape):
    return int(math.prod(shape)) if shape else 1


def is_tensor(a):
    return isinstance(a, dict) and a.get("type") == "tensor"


def tensors(args):
    """Every tensor description, flattening list / tuple arguments."""
    out = []
    for a in args:
        if is_tensor(a):
            out.append(a)
        elif isinstance(a, dict) and a.get("type") in ("list", "tuple"):
            out.extend(tensors(a.get("value") or []))
    return out


def positional(args):
    return [a for a in args if not a.get("name")]


def named(args, name, default=None):
    for a in args:
        if a.get("name") == name:
            return value(a, default)
    return default


def value(a, default=None):
    if a is None:
        return default
    if a.get("type") in ("list", "tuple"):
        return [value(e, default) for e in (a.get("value") or [])]
    return a.get("value", default)


def arg(args, index, name, default=None):
    """Argument ``name`` given by keyword, else the ``index``-th positional one."""
    v = named(args, name, None)
    if v is not None:
        return v
    pos = positional(args)
    if index < len(pos):
        return value(pos[index], default) if not is_tensor(pos[index]) else pos[index]
    return default


def tbytes(t):
    return numel(t["shape"]) * nbytes_of(t.get("dtype"))


def broadcast(*shapes):
    shapes = [tuple(s) for s in shapes if s is not None]
    if not shapes:
        return ()
    n = max(len(s) for s in shapes)
    out = []
    for i in range(n):
        dims = [s[len(s) - n + i] for s in shapes if len(s) - n + i >= 0]
        big = [d for d in dims if d != 1]
        out.append(max(big) if big else 1)
    return tuple(out)


def as_tuple(v, n):
    """Conv/pool hyper-parameter (int or list) expanded to ``n`` spatial dims."""
    if v is None:
        return None
    if isinstance(v, (list, tuple)):
        v = [x for x in v if x is not None]
        if len(v) == 1:
            return tuple(v) * n
        return tuple(v[-n:]) if len(v) >= n else tuple(v) + (v[-1],) * (n - len(v))
    return (v,) * n


def fmt_shape(shape):
    return "x".join(str(d) for d in shape) if shape else "scalar"
