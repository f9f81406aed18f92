"""Convolutions (reference apex/pyprof/prof/conv.py): conv1d/2d/3d, transposed convs and the
``nn.ConvNd`` modules.  Output extent from stride / padding / dilation; groups divide the
reduction.  Forward FLOPs = 2 * N * K * prod(out) * (C/groups) * prod(kernel); backward
(dgrad + wgrad) = 2x."""
from .base import OpModel
from .utility import arg, as_tuple, fmt_shape, nbytes_of, numel, short


class Conv(OpModel):
    kind = "conv"
    matrix = True
    transposed = False

    def parse(self):
        self.ok = len(self.ts) >= 2
        if not self.ok:
            return
        x, w = self.ts[0], self.ts[1]
        self.dtype = x.get("dtype", "float32")
        nd = len(w["shape"]) - 2
        self.nd = nd
        xs = x["shape"]
        self.n = xs[0] if len(xs) == nd + 2 else 1
        self.c = xs[-nd - 1]
        self.inp = tuple(xs[-nd:])
        self.kernel = tuple(w["shape"][2:])
        self.groups = int(arg(self.args, 6 if not self.transposed else 6, "groups", 1) or 1)
        stride = as_tuple(arg(self.args, 3, "stride", 1), nd)
        pad = arg(self.args, 4, "padding", 0)
        dil = as_tuple(arg(self.args, 5 if not self.transposed else 7, "dilation", 1), nd)
        if isinstance(pad, str):  # 'same' / 'valid'
            pad = tuple((d * (k - 1)) // 2 for d, k in zip(dil, self.kernel)) if pad == "same" else (0,) * nd
        pad = as_tuple(pad, nd)
        if self.transposed:
            self.k = w["shape"][1] * self.groups
            opad = as_tuple(arg(self.args, 5, "output_padding", 0), nd)
            self.out = tuple((i - 1) * s - 2 * p + d * (k - 1) + op + 1
                             for i, s, p, d, k, op in zip(self.inp, stride, pad, dil, self.kernel, opad))
        else:
            self.k = w["shape"][0]
            self.out = tuple((i + 2 * p - d * (k - 1) - 1) // s + 1
                             for i, s, p, d, k in zip(self.inp, stride, pad, dil, self.kernel))
        self.stride, self.pad, self.dil = stride, pad, dil
        self.has_bias = len(self.ts) > 2

    def fwd_flops(self):
        if not self.ok:
            return 0
        if self.transposed:  # each input point scatters C/groups * K * prod(kernel) MACs
            macs = self.n * numel(self.inp) * self.c * (self.k // self.groups) * numel(self.kernel)
        else:
            macs = self.n * numel(self.out) * self.k * (self.c // self.groups) * numel(self.kernel)
        return 2 * macs + (self.n * self.k * numel(self.out) if self.has_bias else 0)

    def fwd_bytes(self):
        if not self.ok:
            return 0
        e = nbytes_of(self.dtype)
        wts = self.k * (self.c // self.groups) * numel(self.kernel)
        return e * (self.n * self.c * numel(self.inp) + wts + self.n * self.k * numel(self.out))

    def bprop_flops(self):
        return 2 * self.fwd_flops()

    def bprop_bytes(self):
        return 2 * self.fwd_bytes()

    def params(self):
        if not self.ok:
            return {}
        p = {"N": self.n, "C": self.c, "K": self.k, "in": fmt_shape(self.inp), "R": fmt_shape(self.kernel),
             "out": fmt_shape(self.out)}
        if any(s != 1 for s in self.stride):
            p["stride"] = fmt_shape(self.stride)
        if self.groups != 1:
            p["g"] = self.groups
        p["type"] = short(self.dtype)
        return p


class ConvTranspose(Conv):
    transposed = True


class ConvModule(Conv):
    """``nn.ConvNd.forward(x)``: hyper-parameters from extra_repr."""

    def parse(self):
        self.ok = False
        rp = _repr(self.rec.get("strRepr", ""))
        if not self.ts or "kernel_size" not in rp:
            return
        x = self.ts[0]
        k_sz = rp["kernel_size"]
        nd = len(k_sz)
        cin, cout = rp["in"], rp["out"]
        self.transposed = "output_padding" in rp or self.rec.get("mod", "").startswith("ConvTranspose")
        self.dtype = x.get("dtype", "float32")
        self.nd = nd
        xs = x["shape"]
        self.n = xs[0] if len(xs) == nd + 2 else 1
        self.c = cin
        self.k = cout
        self.inp = tuple(xs[-nd:])
        self.kernel = tuple(k_sz)
        self.groups = rp.get("groups", (1,))[0]
        self.stride = tuple(rp.get("stride", (1,) * nd))
        self.pad = tuple(rp.get("padding", (0,) * nd))
        self.dil = tuple(rp.get("dilation", (1,) * nd))
        if self.transposed:
            opad = tuple(rp.get("output_padding", (0,) * nd))
            self.out = tuple((i - 1) * s - 2 * p + d * (k - 1) + op + 1
                             for i, s, p, d, k, op in zip(self.inp, self.stride, self.pad, self.dil, self.kernel,
                                                          opad))
        else:
            self.out = tuple((i + 2 * p - d * (k - 1) - 1) // s + 1
                             for i, s, p, d, k in zip(self.inp, self.stride, self.pad, self.dil, self.kernel))
        self.has_bias = rp.get("bias", (1,))[0] != 0
        self.ok = True


def _repr(text):
    """'3, 64, kernel_size=(7, 7), stride=(2, 2), padding=(3, 3), bias=False' -> dict."""
    out = {}
    if not text:
        return out
    parts, depth, cur = [], 0, ""
    for ch in text:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    pos = []
    for p in parts:
        p = p.strip()
        if "=" in p:
            k, v = p.split("=", 1)
            v = v.strip().strip("()")
            if v in ("False", "True"):
                out[k.strip()] = (1 if v == "True" else 0,)
                continue
            try:
                out[k.strip()] = tuple(int(x) for x in v.split(",") if x.strip())
            except ValueError:
                out[k.strip()] = v
        elif p:
            try:
                pos.append(int(p))
            except ValueError:
                pass
    if len(pos) >= 2:
        out["in"], out["out"] = pos[0], pos[1]
    return out


OPS = {"conv1d": Conv, "conv2d": Conv, "conv3d": Conv, "conv_transpose1d": ConvTranspose,
       "conv_transpose2d": ConvTranspose, "conv_transpose3d": ConvTranspose, "convolution": Conv}
MODULES = {"Conv1d": ConvModule, "Conv2d": ConvModule, "Conv3d": ConvModule, "ConvTranspose1d": ConvModule,
           "ConvTranspose2d": ConvModule, "ConvTranspose3d": ConvModule}
