"""Per-op FLOP / byte models (reference apex/pyprof/prof/{blas,conv,pointwise,normalization,
softmax,optim,...}.py).  Each model takes the marker's argument descriptions (shapes, dtypes,
scalars recorded by apex.pyprof.nvtx) and returns (flops, bytes, params-string)."""
import math

_BYTES = {"float32": 4, "float": 4, "float16": 2, "half": 2, "bfloat16": 2, "float64": 8, "int64": 8, "int32": 4,
          "uint8": 1, "int8": 1, "bool": 1, "float8_e4m3fn": 1, "float8_e5m2": 1}


def _tensors(args):
    out = []
    for a in args:
        if a.get("type") == "tensor":
            out.append(a)
        elif a.get("type") in ("list", "tuple"):
            out.extend(_tensors(a.get("value", [])))
    return out


def _n(t):
    return int(math.prod(t["shape"])) if t["shape"] else 1


def _b(t):
    return _n(t) * _BYTES.get(t.get("dtype", "float32"), 4)


def _scalar(args, name, default=None):
    for a in args:
        if a.get("name") == name:
            return a.get("value", default)
    return default


def matmul_like(args):
    ts = _tensors(args)
    if len(ts) < 2:
        return 0, sum(_b(t) for t in ts), ""
    a, b = ts[0]["shape"], ts[1]["shape"]
    if len(a) == 1 or len(b) == 1:
        k = a[-1]
        m = _n(ts[0]) // k
        n = 1 if len(b) == 1 else b[-1]
    else:
        k = a[-1]
        m = _n(ts[0]) // k
        n = b[-1] if b[-2] == k else b[-2]
    flops = 2 * m * n * k
    out_bytes = m * n * _BYTES.get(ts[0].get("dtype"), 4)
    return flops, _b(ts[0]) + _b(ts[1]) + out_bytes, "M={},N={},K={}".format(m, n, k)


def linear(args):
    ts = _tensors(args)
    if len(ts) < 2:
        return matmul_like(args)
    x, w = ts[0], ts[1]
    k = x["shape"][-1]
    m = _n(x) // k
    n = w["shape"][0]
    bias = _n(ts[2]) if len(ts) > 2 else 0
    return 2 * m * n * k + m * n * (1 if bias else 0), _b(x) + _b(w) + m * n * _BYTES.get(x.get("dtype"), 4), \
        "M={},N={},K={}".format(m, n, k)


def conv(args, strrepr=""):
    ts = _tensors(args)
    if len(ts) < 2:
        return 0, sum(_b(t) for t in ts), ""
    x, w = ts[0], ts[1]
    n, c = x["shape"][0], x["shape"][1]
    k = w["shape"][0]
    ksz = int(math.prod(w["shape"][2:]))
    stride = _scalar(args, "stride", 1)
    s = stride[0] if isinstance(stride, (list, tuple)) and stride and not isinstance(stride[0], dict) else 1
    if isinstance(stride, int):
        s = stride
    spatial_out = int(math.prod(x["shape"][2:])) // max(1, s ** (len(x["shape"]) - 2))
    groups = _scalar(args, "groups", 1) or 1
    flops = 2 * n * k * spatial_out * (c // groups) * ksz
    out_bytes = n * k * spatial_out * _BYTES.get(x.get("dtype"), 4)
    return flops, _b(x) + _b(w) + out_bytes, "N={},C={},K={},R*S={},out={}".format(n, c, k, ksz, spatial_out)


def pointwise(args, flops_per_elem=1):
    ts = _tensors(args)
    if not ts:
        return 0, 0, ""
    n = max(_n(t) for t in ts)
    return flops_per_elem * n, sum(_b(t) for t in ts) + max(_b(t) for t in ts), "n={}".format(n)


def norm(args):
    ts = _tensors(args)
    if not ts:
        return 0, 0, ""
    x = ts[0]
    return 8 * _n(x), 2 * _b(x) + sum(_b(t) for t in ts[1:]), "shape={}".format(tuple(x["shape"]))


def softmax(args):
    ts = _tensors(args)
    if not ts:
        return 0, 0, ""
    return 5 * _n(ts[0]), 2 * _b(ts[0]), "shape={}".format(tuple(ts[0]["shape"]))


def sdpa(args):
    ts = _tensors(args)
    if len(ts) < 3:
        return pointwise(args)
    q, k = ts[0]["shape"], ts[1]["shape"]
    d = q[-1]
    sq, sk = q[-2], k[-2]
    bh = _n(ts[0]) // (sq * d)
    return 4 * bh * sq * sk * d, sum(_b(t) for t in ts[:3]) + _b(ts[0]), "BH={},Sq={},Sk={},D={}".format(bh, sq, sk, d)


MODELS = {
    "linear": linear, "matmul": matmul_like, "mm": matmul_like, "bmm": matmul_like, "addmm": linear,
    "baddbmm": matmul_like, "einsum": matmul_like, "__matmul__": matmul_like,
    "conv1d": conv, "conv2d": conv, "conv3d": conv, "conv_transpose2d": conv,
    "layer_norm": norm, "batch_norm": norm, "group_norm": norm, "instance_norm": norm, "rms_norm": norm,
    "softmax": softmax, "log_softmax": softmax, "cross_entropy": softmax,
    "scaled_dot_product_attention": sdpa,
    "relu": pointwise, "gelu": lambda a: pointwise(a, 8), "silu": lambda a: pointwise(a, 4),
    "sigmoid": lambda a: pointwise(a, 4), "tanh": lambda a: pointwise(a, 4), "dropout": pointwise,
    "add": pointwise, "sub": pointwise, "mul": pointwise, "div": pointwise, "__add__": pointwise,
    "__mul__": pointwise, "__iadd__": pointwise, "add_": pointwise, "mul_": pointwise,
}

MODULE_OPS = {"Linear": "linear", "Conv1d": "conv1d", "Conv2d": "conv2d", "Conv3d": "conv3d", "LayerNorm": "layer_norm",
              "BatchNorm2d": "batch_norm", "BatchNorm1d": "batch_norm", "ReLU": "relu", "GELU": "gelu",
              "Softmax": "softmax", "Dropout": "dropout"}


def _repr_ints(text):
    out = {}
    for part in (text or "").split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            try:
                out[k.strip()] = int(v.strip())
            except ValueError:
                pass
    return out


def module_linear(rec):
    """nn.Linear.forward marker: weight shape from extra_repr (in/out features)."""
    ts = _tensors(rec.get("args", []))
    rp = _repr_ints(rec.get("strRepr", ""))
    if not ts or "in_features" not in rp:
        return 0, 0, ""
    x = ts[0]
    k, n = rp["in_features"], rp["out_features"]
    m = _n(x) // k
    eb = _BYTES.get(x.get("dtype"), 4)
    return 2 * m * n * k, (m * k + n * k + m * n) * eb, "M={},N={},K={}".format(m, n, k)


def model_for(rec):
    op, mod = rec.get("op", ""), rec.get("mod", "")
    if op == "forward" and mod == "Linear":
        return module_linear(rec)
    if op == "forward" and mod in MODULE_OPS:
        op = MODULE_OPS[mod]
    fn = MODELS.get(op)
    if fn is None:
        return 0, 0, ""
    if fn is conv:
        return conv(rec.get("args", []), rec.get("strRepr", ""))
    return fn(rec.get("args", []))
