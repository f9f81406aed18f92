"""Optimizer and multi-tensor ops (reference apex/pyprof/prof/optim.py).  ``apex.pyprof.nvtx
.init()`` also annotates the ``apex.amp_C`` multi-tensor entry points, whose markers carry the
whole tensor lists, so every fused optimizer step / unscale / norm is priced from its lists:
bytes = lists read + lists written (one pass), FLOPs = per-element cost x elements."""
from .base import OpModel
from .utility import nbytes_of, numel, tensors

# op -> (flops per element, lists read, lists written); list indices past the call's depth are
# ignored (e.g. the optional model-copy output)
_R4, _W4 = (0, 1, 2, 3), (1, 2, 3, 4)
MT = {
    "multi_tensor_scale": (1, (0,), (1,)), "multi_tensor_scale_t": (1, (0,), (1,)),
    "multi_tensor_axpby": (3, (0, 1), (2,)), "multi_tensor_check_finite": (1, (0,), ()),
    "multi_tensor_l2norm": (2, (0,), ()), "multi_tensor_l2norm_mp": (2, (0,), ()),
    "multi_tensor_maxnorm": (1, (0,), ()), "multi_tensor_l2norm_scale": (3, (0,), (1,)),
    "multi_tensor_norm_out": (2, (0,), ()), "multi_tensor_adam": (18, _R4, _W4),
    "multi_tensor_adam_capturable": (18, _R4, _W4), "multi_tensor_adam_undo": (20, _R4, _W4),
    "multi_tensor_sgd": (5, (0, 1, 2), (1, 2, 3)), "multi_tensor_sgd_capturable": (5, (0, 1, 2), (1, 2, 3)),
    "multi_tensor_adagrad": (8, (0, 1, 2), (1, 2)), "multi_tensor_novograd": (12, (0, 1, 2), (1, 2)),
    "multi_tensor_lamb": (24, _R4, _W4), "multi_tensor_lamb_mp": (24, _R4, _W4),
    "multi_tensor_lamb_stage1_cuda": (16, (0, 1, 2, 3), (2, 3, 4)),
    "multi_tensor_lamb_stage2_cuda": (3, (0, 1), (0, 2)), "multi_tensor_cast": (0, (0,), (1,)),
}


class MultiTensor(OpModel):
    kind = "optim"

    def parse(self):
        self.name = self.rec.get("op", "")
        self.lists = []
        for a in self.args:  # the tensor_lists argument: a list of lists of tensors
            if a.get("type") in ("list", "tuple") and a.get("value") and \
                    all(v.get("type") in ("list", "tuple") for v in a["value"]):
                self.lists = [tensors(v.get("value") or []) for v in a["value"]]
                break
        self.n = sum(numel(t["shape"]) for t in self.lists[0]) if self.lists else 0

    def fwd_flops(self):
        return MT.get(self.name, (1, (), ()))[0] * self.n

    def fwd_bytes(self):
        _, reads, writes = MT.get(self.name, (1, tuple(range(len(self.lists))), ()))
        total = 0
        for i, lst in enumerate(self.lists):
            b = sum(numel(t["shape"]) * nbytes_of(t.get("dtype")) for t in lst)
            total += b * ((i in reads) + (i in writes))
        return total

    def params(self):
        return {"lists": len(self.lists), "tensors": len(self.lists[0]) if self.lists else 0, "n": self.n}


OPS = {name: MultiTensor for name in MT}
MODULES = {}
