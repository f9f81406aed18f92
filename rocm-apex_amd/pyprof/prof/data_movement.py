"""Indexing, slicing, joining, mutation, random sampling and recurrent cells (reference
apex/pyprof/prof/index_slice_join_mutate.py, randomSample.py, recurrentCell.py, misc.py).
Views (reshape / permute / transpose / expand / slicing) move no data and report 0 bytes;
materialising ops (cat, contiguous, clone, gather, index_select...) read their input once
and write their output once."""
from .base import OpModel
from .utility import arg, fmt_shape, nbytes_of, numel, short

VIEWS = {"view", "view_as", "reshape", "reshape_as", "permute", "transpose", "t", "expand", "expand_as", "unsqueeze",
         "squeeze", "flatten", "unflatten", "narrow", "select", "unbind", "split", "chunk", "tensor_split",
         "__getitem__", "as_strided", "detach", "movedim", "swapaxes", "unfold", "diagonal", "real", "imag",
         "contiguous_noop", "numpy", "split_with_sizes"}


class DataMove(OpModel):
    kind = "data"

    def parse(self):
        self.name = self.rec.get("op", "")
        x = self.ts[0] if self.ts else {"shape": (), "dtype": "float32"}
        self.dtype = x.get("dtype", "float32")
        self.n_in = sum(numel(t["shape"]) for t in self.ts)
        self.shape = tuple(x["shape"])
        name = self.name.rstrip("_")
        if name in ("cat", "concat", "concatenate", "stack", "hstack", "vstack", "dstack"):
            self.n_out = self.n_in
        elif name == "index_select":
            dim = arg(self.args, 1, "dim", 0)
            extent = self.shape[dim] if self.shape and isinstance(dim, int) else 1
            self.n_out = numel(self.shape) // max(1, extent) * numel(self.ts[-1]["shape"])
        elif name in ("gather", "take", "masked_select", "take_along_dim"):
            self.n_out = numel(self.ts[-1]["shape"])
        elif name in ("repeat", "tile", "repeat_interleave"):
            reps = arg(self.args, 1, "repeats", 1)
            r = numel(reps) if isinstance(reps, (list, tuple)) else (reps if isinstance(reps, int) else 1)
            self.n_out = numel(self.shape) * r
        elif name in ("zero", "fill", "zeros_like", "ones_like", "full_like", "empty_like", "new_zeros", "new_ones"):
            self.n_out, self.n_in = numel(self.shape), 0
        else:  # clone, contiguous, copy, flip, roll, scatter, index_put, masked_fill, where-like
            self.n_out = numel(self.shape)

    def fwd_flops(self):
        return 0

    def fwd_bytes(self):
        if self.name in VIEWS:
            return 0
        e = nbytes_of(self.dtype)
        return (self.n_in + self.n_out) * e

    def params(self):
        return {"T": fmt_shape(self.shape), "type": short(self.dtype)}


class Random(OpModel):
    """rand / randn / normal_ / uniform_ / bernoulli / randint / randperm / multinomial: the
    output is written once; Philox draws priced as a few FLOPs per value."""
    kind = "random"

    def parse(self):
        self.name = self.rec.get("op", "")
        if self.ts:
            self.shape = tuple(self.ts[0]["shape"])
            self.dtype = self.ts[0].get("dtype", "float32")
        else:
            size = [a.get("value") for a in self.args if a.get("type") == "int"]
            lst = [a for a in self.args if a.get("type") in ("list", "tuple")]
            if lst:
                size = [e.get("value") for e in lst[0].get("value", []) if isinstance(e.get("value"), int)]
            self.shape = tuple(size)
            self.dtype = next((a.get("value") for a in self.args if a.get("type") == "dtype"), "float32")

    def fwd_flops(self):
        return 8 * numel(self.shape)

    def fwd_bytes(self):
        return numel(self.shape) * nbytes_of(self.dtype)

    def params(self):
        return {"T": fmt_shape(self.shape), "type": short(self.dtype)}


class RecurrentCell(OpModel):
    """``nn.LSTMCell`` / ``GRUCell`` / ``RNNCell`` forward: gate GEMMs (input and hidden) plus
    the gate pointwise math."""
    kind = "rnn"
    matrix = True
    GATES = {"LSTMCell": 4, "GRUCell": 3, "RNNCell": 1, "LSTM": 4, "GRU": 3, "RNN": 1}

    def parse(self):
        mod = self.rec.get("mod", "")
        self.gates = self.GATES.get(mod, 1)
        parts = [p.strip() for p in (self.rec.get("strRepr") or "").split(",")]
        ints = [int(p) for p in parts if p.isdigit()]
        x = self.ts[0] if self.ts else {"shape": (1, 1), "dtype": "float32"}
        self.dtype = x.get("dtype", "float32")
        self.inp = ints[0] if ints else x["shape"][-1]
        self.hid = ints[1] if len(ints) > 1 else self.inp
        self.rows = numel(x["shape"][:-1])

    def fwd_flops(self):
        gemm = 2 * self.rows * (self.inp + self.hid) * self.gates * self.hid
        return gemm + 10 * self.rows * self.gates * self.hid

    def fwd_bytes(self):
        e = nbytes_of(self.dtype)
        w = (self.inp + self.hid) * self.gates * self.hid
        return e * (w + self.rows * (self.inp + 2 * self.hid) + self.rows * self.hid * 2)

    def bprop_flops(self):
        return 2 * self.fwd_flops()

    def params(self):
        return {"rows": self.rows, "in": self.inp, "hid": self.hid, "gates": self.gates, "type": short(self.dtype)}


OPS = {}
for _op in list(VIEWS) + ["cat", "concat", "concatenate", "stack", "hstack", "vstack", "dstack", "index_select",
                          "gather", "take", "masked_select", "take_along_dim", "repeat", "tile", "repeat_interleave",
                          "zero_", "fill_", "zeros_like", "ones_like", "full_like", "empty_like", "new_zeros",
                          "new_ones", "clone", "contiguous", "copy", "flip", "roll", "scatter", "scatter_",
                          "scatter_add", "scatter_add_", "index_put", "index_put_", "index_add", "index_add_",
                          "index_copy", "index_copy_", "masked_fill", "masked_fill_", "masked_scatter",
                          "masked_scatter_", "nonzero", "tril", "triu", "pad", "interpolate", "upsample",
                          "pixel_shuffle", "pixel_unshuffle", "one_hot", "unique", "bincount", "histc"]:
    OPS[_op] = DataMove
for _op in ("rand", "randn", "randint", "randperm", "rand_like", "randn_like", "randint_like", "normal", "normal_",
            "uniform_", "bernoulli", "bernoulli_", "multinomial", "exponential_", "geometric_", "log_normal_",
            "cauchy_", "random_", "poisson"):
    OPS[_op] = Random
MODULES = {m: RecurrentCell for m in RecurrentCell.GATES}
