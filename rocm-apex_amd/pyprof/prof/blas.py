"""GEMM-shaped ops (reference apex/pyprof/prof/blas.py, linear.py): addmm, mm, bmm, baddbmm,
addbmm, matmul / @, mv / addmv, dot, linear, einsum and the module ``nn.Linear``.

Forward FLOPs = 2*M*N*K (+ M*N for a bias / beta*C); backward = dgrad + wgrad = 2x that."""
import re

from .base import OpModel
from .utility import arg, fmt_shape, named, nbytes_of, numel, short


class Gemm(OpModel):
    kind = "blas"
    matrix = True

    def parse(self):
        self.batch, self.m, self.n, self.k = 1, 0, 0, 0
        self.bias = False
        self.dtype = self.ts[0].get("dtype", "float32") if self.ts else "float32"
        op = self.rec.get("op", "")
        ts = self.ts
        try:
            getattr(self, "_shape_" + self.family(op))(ts)
        except (IndexError, KeyError, ValueError, ZeroDivisionError, TypeError):
            self.m = self.n = self.k = 0

    @staticmethod
    def family(op):
        op = op.rstrip("_")
        if op in ("addmm", "baddbmm", "addbmm", "addmv"):
            return op
        if op in ("mm", "bmm", "mv", "dot", "vdot", "inner", "outer", "ger"):
            return op if op not in ("vdot", "inner") else "dot"
        if op == "linear":
            return "linear"
        return "matmul"  # matmul, __matmul__, __rmatmul__

    def _shape_addmm(self, ts):
        c, a, b = ts[0], ts[1], ts[2]
        self.m, self.k = a["shape"][-2], a["shape"][-1]
        self.n = b["shape"][-1]
        self.bias = named(self.args, "beta", 1) != 0

    def _shape_baddbmm(self, ts):
        c, a, b = ts[0], ts[1], ts[2]
        self.batch, self.m, self.k = a["shape"]
        self.n = b["shape"][-1]
        self.bias = named(self.args, "beta", 1) != 0

    def _shape_addbmm(self, ts):
        self._shape_baddbmm(ts)

    def _shape_addmv(self, ts):
        a = ts[1]
        self.m, self.k, self.n = a["shape"][0], a["shape"][1], 1
        self.bias = True

    def _shape_mm(self, ts):
        a, b = ts[0], ts[1]
        self.m, self.k = a["shape"]
        self.n = b["shape"][1]

    def _shape_bmm(self, ts):
        a, b = ts[0], ts[1]
        self.batch, self.m, self.k = a["shape"]
        self.n = b["shape"][2]

    def _shape_mv(self, ts):
        a = ts[0]
        self.m, self.k, self.n = a["shape"][0], a["shape"][1], 1

    def _shape_dot(self, ts):
        self.m, self.n, self.k = 1, 1, ts[0]["shape"][0]

    def _shape_outer(self, ts):
        self.m, self.n, self.k = ts[0]["shape"][0], ts[1]["shape"][0], 1

    _shape_ger = _shape_outer

    def _shape_linear(self, ts):
        x, w = ts[0], ts[1]
        self.k = x["shape"][-1]
        self.m = numel(x["shape"]) // max(1, self.k)
        self.n = w["shape"][0]
        self.bias = len(ts) > 2

    def _shape_matmul(self, ts):
        a, b = ts[0]["shape"], ts[1]["shape"]
        if len(a) == 1 and len(b) == 1:
            return self._shape_dot(ts)
        if len(b) == 1:  # matrix-vector (batched)
            self.k, self.n = b[0], 1
            self.m = numel(a) // self.k
            return
        if len(a) == 1:
            self.m, self.k, self.n = 1, a[0], b[-1]
            self.batch = numel(b[:-2])
            return
        self.m, self.k, self.n = a[-2], a[-1], b[-1]
        self.batch = max(numel(a[:-2]), numel(b[:-2]))

    # ---- costs ----
    def fwd_flops(self):
        f = 2 * self.batch * self.m * self.n * self.k
        return f + (self.batch * self.m * self.n if self.bias else 0)

    def fwd_bytes(self):
        e = nbytes_of(self.dtype)
        b = self.batch
        io = b * (self.m * self.k + self.k * self.n + self.m * self.n)
        return e * (io + (b * self.m * self.n if self.bias else 0))

    def bprop_flops(self):
        return 2 * 2 * self.batch * self.m * self.n * self.k

    def bprop_bytes(self):
        return 2 * self.fwd_bytes()

    def params(self):
        p = {"M": self.m, "N": self.n, "K": self.k}
        if self.batch > 1:
            p["B"] = self.batch
        p["type"] = short(self.dtype)
        return p


class LinearModule(Gemm):
    """``nn.Linear.forward``: the weight shape comes from the module's extra_repr."""

    def parse(self):
        self.batch, self.bias = 1, False
        self.dtype = self.ts[0].get("dtype", "float32") if self.ts else "float32"
        rp = {}
        for part in (self.rec.get("strRepr") or "").split(","):
            if "=" in part:
                k, v = part.split("=", 1)
                rp[k.strip()] = v.strip()
        try:
            self.k, self.n = int(rp["in_features"]), int(rp["out_features"])
            self.m = numel(self.ts[0]["shape"]) // self.k
            self.bias = rp.get("bias", "True") == "True"
        except (KeyError, ValueError, IndexError, ZeroDivisionError):
            self.m = self.n = self.k = 0


class Einsum(OpModel):
    """FLOPs = 2 * product of every distinct index extent (one multiply-add per point of the
    joint iteration space); bytes = operands + output."""
    kind = "blas"
    matrix = True

    def parse(self):
        eq = arg(self.args, 0, "equation", "")
        self.eq = eq if isinstance(eq, str) else ""
        self.space = 0
        self.out = 0
        try:
            lhs, _, rhs = self.eq.replace(" ", "").partition("->")
            extents = {}
            for spec, t in zip(lhs.split(","), self.ts):
                letters = [c for c in spec if c.isalpha()]
                for c, d in zip(letters, t["shape"][-len(letters):] if letters else []):
                    extents[c] = max(extents.get(c, 1), d)
            self.space = numel(list(extents.values()))
            self.out = numel([extents.get(c, 1) for c in rhs if c.isalpha()])
        except (ValueError, KeyError):
            pass

    def fwd_flops(self):
        return 2 * self.space

    def fwd_bytes(self):
        e = nbytes_of(self.ts[0].get("dtype")) if self.ts else 4
        return sum(numel(t["shape"]) for t in self.ts) * e + self.out * e

    def bprop_flops(self):
        return 2 * self.fwd_flops()

    def params(self):
        return {"eq": re.sub(r"[,\s]", ";", self.eq), "shapes": "|".join(fmt_shape(t["shape"]) for t in self.ts)}


OPS = {}
for _name in ("addmm", "addmm_", "mm", "bmm", "baddbmm", "baddbmm_", "addbmm", "addbmm_", "matmul", "__matmul__",
              "__rmatmul__", "mv", "addmv", "addmv_", "dot", "vdot", "inner", "outer", "ger", "linear"):
    OPS[_name] = Gemm
OPS["einsum"] = Einsum
MODULES = {"Linear": LinearModule, "LazyLinear": LinearModule, "Bilinear": Gemm}
