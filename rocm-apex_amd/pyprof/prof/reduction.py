"""Reductions, softmax and losses (reference apex/pyprof/prof/reduction.py, softmax.py,
loss.py).  A reduction reads its input once and writes the reduced output; softmax reads
twice-ish (max + sum passes fused) and writes once; losses are priced as their elementwise
part plus a reduction."""
from .base import OpModel
from .utility import arg, fmt_shape, nbytes_of, numel, short


def _reduced_shape(shape, dim, keepdim):
    if dim is None or dim == [] or dim == ():
        return (1,) * len(shape) if keepdim else ()
    dims = dim if isinstance(dim, (list, tuple)) else [dim]
    dims = {d % max(1, len(shape)) for d in dims if isinstance(d, int)}
    return tuple((1 if i in dims else s) for i, s in enumerate(shape) if keepdim or i not in dims)


class Reduction(OpModel):
    kind = "reduction"
    COST = {"sum": 1, "mean": 1, "nansum": 2, "nanmean": 2, "prod": 1, "norm": 2, "var": 3, "std": 3,
            "var_mean": 3, "std_mean": 3, "max": 1, "min": 1, "amax": 1, "amin": 1, "argmax": 1, "argmin": 1,
            "aminmax": 2, "logsumexp": 6, "cumsum": 1, "cumprod": 1, "all": 1, "any": 1, "count_nonzero": 1,
            "linalg_vector_norm": 2, "vector_norm": 2, "median": 4, "mode": 4, "topk": 4, "sort": 8, "argsort": 8,
            "kthvalue": 4}

    def parse(self):
        op = self.rec.get("op", "").rstrip("_")
        self.name = op
        x = self.ts[0] if self.ts else {"shape": (), "dtype": "float32"}
        self.inp = tuple(x["shape"])
        self.dtype = x.get("dtype", "float32")
        dim = arg(self.args, 1, "dim", None)
        if isinstance(dim, dict):  # a tensor in the dim slot (e.g. torch.max(a, b)) -> binary
            dim = None
        keep = bool(arg(self.args, 2, "keepdim", False)) if not isinstance(arg(self.args, 2, "keepdim", False),
                                                                              dict) else False
        self.out = self.inp if op in ("cumsum", "cumprod", "sort", "argsort") else \
            _reduced_shape(self.inp, dim, keep)

    def fwd_flops(self):
        return self.COST.get(self.name, 1) * numel(self.inp)

    def fwd_bytes(self):
        return (numel(self.inp) + numel(self.out)) * nbytes_of(self.dtype)

    def bprop_flops(self):
        return numel(self.inp)

    def bprop_bytes(self):
        return (numel(self.inp) + numel(self.out)) * nbytes_of(self.dtype)

    def params(self):
        return {"T": fmt_shape(self.inp), "out": fmt_shape(self.out), "type": short(self.dtype)}


class Softmax(OpModel):
    kind = "softmax"

    def parse(self):
        x = self.ts[0] if self.ts else {"shape": (), "dtype": "float32"}
        self.shape = tuple(x["shape"])
        self.dtype = x.get("dtype", "float32")
        self.out_dtype = arg(self.args, 3, "dtype", None) or self.dtype
        self.masked = len(self.ts) > 1  # apex scaled_masked_softmax / masked_fill fusions

    def fwd_flops(self):
        return 5 * numel(self.shape)  # max, sub, exp, sum, div

    def fwd_bytes(self):
        n = numel(self.shape)
        extra = numel(self.ts[1]["shape"]) * nbytes_of(self.ts[1].get("dtype")) if self.masked else 0
        return n * (nbytes_of(self.dtype) + nbytes_of(self.out_dtype)) + extra

    def bprop_flops(self):
        return 4 * numel(self.shape)  # dy*y, row-sum, sub, mul

    def bprop_bytes(self):
        return 3 * numel(self.shape) * nbytes_of(self.dtype)

    def params(self):
        return {"T": fmt_shape(self.shape), "type": short(self.dtype)}


class Loss(OpModel):
    kind = "loss"
    COST = {"mse_loss": 3, "l1_loss": 3, "smooth_l1_loss": 5, "huber_loss": 5, "binary_cross_entropy": 8,
            "binary_cross_entropy_with_logits": 12, "kl_div": 6, "nll_loss": 1, "cross_entropy": 7,
            "poisson_nll_loss": 6, "soft_margin_loss": 8, "hinge_embedding_loss": 3, "margin_ranking_loss": 4,
            "cosine_embedding_loss": 6, "multilabel_soft_margin_loss": 10, "triplet_margin_loss": 8,
            "ctc_loss": 20, "gaussian_nll_loss": 8, "multi_margin_loss": 4}

    def parse(self):
        op = self.rec.get("op", "")
        if op == "forward":
            mod = self.rec.get("mod", "")
            op = {"MSELoss": "mse_loss", "L1Loss": "l1_loss", "CrossEntropyLoss": "cross_entropy",
                  "NLLLoss": "nll_loss", "BCELoss": "binary_cross_entropy", "KLDivLoss": "kl_div",
                  "BCEWithLogitsLoss": "binary_cross_entropy_with_logits", "SmoothL1Loss": "smooth_l1_loss",
                  "HuberLoss": "huber_loss", "CTCLoss": "ctc_loss"}.get(mod, mod.lower())
        self.name = op
        x = self.ts[0] if self.ts else {"shape": (), "dtype": "float32"}
        self.shape = tuple(x["shape"])
        self.dtype = x.get("dtype", "float32")

    def fwd_flops(self):
        return self.COST.get(self.name, 4) * numel(self.shape)

    def fwd_bytes(self):
        return sum(numel(t["shape"]) * nbytes_of(t.get("dtype")) for t in self.ts) + nbytes_of(self.dtype)

    def bprop_bytes(self):
        return self.fwd_bytes() + numel(self.shape) * nbytes_of(self.dtype)

    def params(self):
        return {"T": fmt_shape(self.shape), "type": short(self.dtype)}


OPS = {}
for _op in Reduction.COST:
    OPS[_op] = Reduction
for _op in ("softmax", "log_softmax", "softmin", "_softmax", "scaled_masked_softmax", "scaled_softmax",
            "scaled_upper_triang_masked_softmax", "gumbel_softmax"):
    OPS[_op] = Softmax
for _op in Loss.COST:
    OPS[_op] = Loss
MODULES = {"Softmax": Softmax, "LogSoftmax": Softmax, "Softmin": Softmax, "FusedScaleMaskSoftmax": Softmax}
for _m in ("MSELoss", "L1Loss", "CrossEntropyLoss", "NLLLoss", "BCELoss", "KLDivLoss", "BCEWithLogitsLoss",
           "SmoothL1Loss", "HuberLoss", "CTCLoss"):
    MODULES[_m] = Loss
