"""Normalization, pooling and embedding (reference apex/pyprof/prof/normalization.py,
pooling.py, embedding.py).  Normalizations read x, write y (+ per-channel statistics);
backward reads x, dy and writes dx.  Pooling output extent follows kernel / stride / padding."""
from .base import OpModel
from .utility import arg, as_tuple, fmt_shape, nbytes_of, numel, short


class Norm(OpModel):
    kind = "normalization"

    def parse(self):
        op = self.rec.get("op", "")
        if op == "forward":
            op = self.rec.get("mod", "")
        self.name = op
        x = self.ts[0] if self.ts else {"shape": (), "dtype": "float32"}
        self.shape = tuple(x["shape"])
        self.dtype = x.get("dtype", "float32")
        self.affine = sum(numel(t["shape"]) * nbytes_of(t.get("dtype")) for t in self.ts[1:])

    def fwd_flops(self):
        return 8 * numel(self.shape)  # mean, var (two passes of mul-add) + normalize + affine

    def fwd_bytes(self):
        return 2 * numel(self.shape) * nbytes_of(self.dtype) + self.affine

    def bprop_flops(self):
        return 12 * numel(self.shape)

    def bprop_bytes(self):
        return 3 * numel(self.shape) * nbytes_of(self.dtype) + 2 * self.affine

    def params(self):
        return {"T": fmt_shape(self.shape), "type": short(self.dtype)}


class Pool(OpModel):
    kind = "pooling"

    def parse(self):
        op = self.rec.get("op", "")
        self.name = op
        x = self.ts[0] if self.ts else {"shape": (), "dtype": "float32"}
        self.dtype = x.get("dtype", "float32")
        xs = tuple(x["shape"])
        nd = 3 if "3d" in op else (1 if "1d" in op else 2)
        nd = min(nd, max(1, len(xs) - 1))
        self.lead, self.inp = xs[:-nd], xs[-nd:]
        if op.startswith("adaptive"):
            size = as_tuple(arg(self.args, 1, "output_size", 1), nd)
            self.out = tuple(o if o is not None else i for o, i in zip(size, self.inp))
            self.window = tuple(max(1, -(-i // o)) for i, o in zip(self.inp, self.out))
        else:
            k = as_tuple(arg(self.args, 1, "kernel_size", 1), nd)
            s = as_tuple(arg(self.args, 2, "stride", None) or k, nd)
            p = as_tuple(arg(self.args, 3, "padding", 0), nd)
            d = as_tuple(arg(self.args, 4, "dilation", 1), nd) if op.startswith("max") else (1,) * nd
            ceil = bool(arg(self.args, 5, "ceil_mode", False))
            self.out = tuple(((i + 2 * pp - dd * (kk - 1) - 1 + (ss - 1 if ceil else 0)) // ss) + 1
                             for i, kk, ss, pp, dd in zip(self.inp, k, s, p, d))
            self.window = k

    def fwd_flops(self):
        return numel(self.lead) * numel(self.out) * numel(self.window)

    def fwd_bytes(self):
        return numel(self.lead) * (numel(self.inp) + numel(self.out)) * nbytes_of(self.dtype)

    def bprop_bytes(self):
        return numel(self.lead) * (numel(self.inp) + 2 * numel(self.out)) * nbytes_of(self.dtype)

    def params(self):
        return {"in": fmt_shape(self.lead + self.inp), "out": fmt_shape(self.out), "k": fmt_shape(self.window),
                "type": short(self.dtype)}


class Embedding(OpModel):
    kind = "embedding"

    def parse(self):
        self.idx = self.ts[0] if self.ts else {"shape": (), "dtype": "int64"}
        self.w = self.ts[1] if len(self.ts) > 1 else {"shape": (1, 1), "dtype": "float32"}
        self.dim = self.w["shape"][-1] if self.w["shape"] else 1

    def fwd_flops(self):
        return 0

    def fwd_bytes(self):
        n = numel(self.idx["shape"])
        return n * nbytes_of(self.idx.get("dtype")) + 2 * n * self.dim * nbytes_of(self.w.get("dtype"))

    def bprop_flops(self):  # scatter-add of the rows
        return numel(self.idx["shape"]) * self.dim

    def params(self):
        return {"I": fmt_shape(self.idx["shape"]), "E": fmt_shape(self.w["shape"]),
                "type": short(self.w.get("dtype"))}


OPS = {"batch_norm": Norm, "layer_norm": Norm, "group_norm": Norm, "instance_norm": Norm, "rms_norm": Norm,
       "local_response_norm": Norm, "normalize": Norm, "fused_layer_norm": Norm, "fused_rms_norm": Norm,
       "native_layer_norm": Norm, "native_batch_norm": Norm, "embedding": Embedding, "embedding_bag": Embedding}
for _p in ("max_pool1d", "max_pool2d", "max_pool3d", "avg_pool1d", "avg_pool2d", "avg_pool3d", "lp_pool1d",
           "lp_pool2d", "adaptive_avg_pool1d", "adaptive_avg_pool2d", "adaptive_avg_pool3d", "adaptive_max_pool1d",
           "adaptive_max_pool2d", "adaptive_max_pool3d", "max_pool1d_with_indices", "max_pool2d_with_indices"):
    OPS[_p] = Pool
MODULES = {m: Norm for m in ("BatchNorm1d", "BatchNorm2d", "BatchNorm3d", "SyncBatchNorm", "LayerNorm", "GroupNorm",
                             "InstanceNorm1d", "InstanceNorm2d", "InstanceNorm3d", "RMSNorm", "LocalResponseNorm",
                             "FusedLayerNorm", "FusedRMSNorm", "MixedFusedLayerNorm", "BatchNorm2d_NHWC")}
