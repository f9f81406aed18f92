"""Op model base (reference apex/pyprof/prof/base.py OperatorLayerBase).

An op model reads one parsed kernel record (its marker's argument descriptions, direction and
kernel name) and reports FLOPs (FMA = 2), DRAM bytes (compulsory traffic: inputs read once,
outputs written once), a parameter string and whether the kernel is a matrix-core (MFMA) kernel.

Direction: a backward (``dir == 'bprop'``) record is priced by ``bprop_flops`` /
``bprop_bytes``, which default to the forward cost (pointwise and data-movement ops) and are
overridden by GEMM-shaped ops (dgrad + wgrad = 2x the forward FLOPs)."""
from .utility import positional, tbytes, tensors

# gfx950 kernel names that run on matrix cores: hipBLASLt/Tensile ("Cijk_..._MT"), composable
# kernel XDL pipelines, MIOpen implicit GEMM, and this package's MFMA kernels
MFMA_HINTS = ("Cijk_", "_MT", "xdl", "Xdl", "XDL", "mfma", "MFMA", "igemm", "Igemm", "gemm_mfma", "gemm256",
              "flash", "fmha", "conv_igemm", "fprop_kernel", "wgrad_kernel")


class OpModel(object):
    kind = "misc"
    matrix = False  # GEMM-shaped: the tc column is meaningful

    def __init__(self, rec):
        self.rec = rec
        self.args = rec.get("args", []) or []
        self.pos = positional(self.args)
        self.ts = tensors(self.args)
        self.dir = rec.get("dir") or "fprop"
        self.kname = rec.get("kName", "") or ""
        self.parse()

    # ---- to override ----
    def parse(self):
        pass

    def fwd_flops(self):
        return 0

    def fwd_bytes(self):
        return sum(tbytes(t) for t in self.ts)

    def bprop_flops(self):
        return self.fwd_flops()

    def bprop_bytes(self):
        return self.fwd_bytes()

    def params(self):
        return {}

    # ---- public ----
    def flops(self):
        return int(self.bprop_flops() if self.dir == "bprop" else self.fwd_flops())

    def bytes(self):
        return int(self.bprop_bytes() if self.dir == "bprop" else self.fwd_bytes())

    def tc(self):
        if not self.matrix:
            return "-"
        return 1 if any(h in self.kname for h in MFMA_HINTS) else 0

    def op(self):
        return self.rec.get("op", "")

    def mod(self):
        return self.rec.get("mod", "")


def param_string(params):
    return ",".join("{}={}".format(k, v) for k, v in params.items())
