"""``amp_C``: the multi-tensor op namespace (reference csrc/amp_C_frontend.cpp:147-174).

GPU tensor lists run on the gfx950 kernels of the native extension (``_C.amp_C``); CPU lists
run the torch reference implementations (:mod:`apex.ops.multi_tensor_ref`).  Dispatch is
per call on the device of the first tensor, so one name works in both tiers.
"""
import torch

from . import _native
from .ops import multi_tensor_ref as _ref

__all__ = [
    "multi_tensor_scale", "multi_tensor_scale_t", "multi_tensor_axpby", "multi_tensor_check_finite",
    "multi_tensor_l2norm", "multi_tensor_l2norm_mp", "multi_tensor_maxnorm", "multi_tensor_l2norm_scale",
    "multi_tensor_norm_out", "multi_tensor_adam", "multi_tensor_adam_capturable", "multi_tensor_adam_undo", "multi_tensor_sgd",
    "multi_tensor_sgd_capturable", "multi_tensor_adagrad", "multi_tensor_novograd", "multi_tensor_lamb",
    "multi_tensor_lamb_mp", "multi_tensor_lamb_stage1_cuda", "multi_tensor_lamb_stage2_cuda",
    "multi_tensor_lamb_stage1_capturable", "multi_tensor_lamb_stage2_capturable", "multi_tensor_cast", "amp_update_scale_", "mta_cache_clear", "mta_cache_size",
]


def _first_tensor(args):
    for a in args:
        if isinstance(a, (list, tuple)):
            for l in a:
                if isinstance(l, (list, tuple)) and l:
                    return l[0]
    return None


def _validate_lists(name, args):
    """Same contract as the native engine (csrc/bindings/mta_host.cpp): every list is
    dtype-homogeneous, so CPU tests catch callers that would corrupt data on the GPU."""
    for a in args:
        if isinstance(a, (list, tuple)) and a and isinstance(a[0], (list, tuple)):
            for d, lst in enumerate(a):
                ts = [x for x in lst if isinstance(x, torch.Tensor)]
                if ts and any(x.dtype != ts[0].dtype for x in ts):
                    raise RuntimeError(f"{name}: list {d} mixes dtypes "
                                       f"({sorted({str(x.dtype) for x in ts})}); split lists by dtype")
            return


def _make(name):
    ref = getattr(_ref, name)

    def op(*args, **kwargs):
        t = _first_tensor(args)
        if t is None:  # state-only ops (amp_update_scale_) take plain tensors
            for a in args:
                if hasattr(a, "is_cuda"):
                    t = a
                    break
        _validate_lists(name, args)
        if _native.use_native(t):
            return getattr(_native.require(f"amp_C.{name}").amp_C, name)(*args, **kwargs)
        with torch.no_grad():
            return ref(*args, **kwargs)

    op.__name__ = name
    op.__doc__ = ref.__doc__
    return op


for _n in __all__:
    globals()[_n] = _make(_n)


def mta_cache_clear():  # noqa: F811
    m = _native.submodule("amp_C")
    if m is not None:
        m.mta_cache_clear()


def mta_cache_size():  # noqa: F811
    m = _native.submodule("amp_C")
    return m.mta_cache_size() if m is not None else 0
