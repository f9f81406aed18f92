"""Loader for the package's HIP extension (``_C``, built by ``tools/build_native.py``).

Policy: GPU tensors ALWAYS go through the native gfx950 kernels.  If the extension is missing
and a GPU op is requested we raise (no silent eager fallback); CPU tensors use the torch
reference implementations in :mod:`apex.ops` (that is what the CPU test tier exercises).
Set ``APEX_AMD_ALLOW_FALLBACK=1`` to permit the torch path on GPU for debugging.
"""
import contextlib
import importlib
import os

_C = None
import_error = None
try:
    _variant = os.environ.get("APEX_AMD_NATIVE_SO")  # A/B experiments: a variant build's .so
    if _variant:
        import importlib.util
        import sys

        _spec = importlib.util.spec_from_file_location(__package__ + "._C", _variant)
        _C = importlib.util.module_from_spec(_spec)
        _spec.loader.exec_module(_C)
        sys.modules[__package__ + "._C"] = _C
    else:
        _C = importlib.import_module(__package__ + "._C")
except Exception as e:  # pragma: no cover - depends on build state
    _C = None
    import_error = e

ALLOW_FALLBACK = os.environ.get("APEX_AMD_ALLOW_FALLBACK", "0") == "1"


def available() -> bool:
    return _C is not None


def require(what: str = "native op"):
    """Return the extension or raise loudly."""
    if _C is None:
        raise RuntimeError(
            f"apex (gfx950) native extension is not built but {what} was requested on a GPU tensor; "
            f"run `python tools/build_native.py` (import error: {import_error!r})")
    return _C


def submodule(name: str):
    if _C is None:
        return None
    return getattr(_C, name, None)


_force_reference = False


@contextlib.contextmanager
def reference_mode(enabled=True):
    """Route GPU tensors through the torch reference implementations (``apex.ops``) inside the
    block.  Parity harness only: tests run one training loop on the HIP kernels and once more
    on the reference ops on the same device and bound the difference."""
    global _force_reference
    prev, _force_reference = _force_reference, bool(enabled)
    try:
        yield
    finally:
        _force_reference = prev


def use_native(*tensors) -> bool:
    """True when the op must run on the HIP path (any GPU tensor among the inputs)."""
    if _force_reference:
        return False
    for t in tensors:
        if t is not None and getattr(t, "is_cuda", False):
            if _C is None and ALLOW_FALLBACK:
                return False
            return True
    return False


def column_sum(x, out_dtype):
    """Sum of a [..., N] tensor over all leading dims (fp32 accumulation) in ``out_dtype``: the bias
    gradient of a dense layer.  The gfx950 two-stage column reduction (deterministic, fixed order)
    for contiguous fp16/bf16/fp32 GPU tensors with N % 8 == 0, torch otherwise."""
    import torch

    if (use_native(x) and submodule("gemm") is not None and x.dim() >= 2 and x.is_contiguous()
            and x.shape[-1] % 8 == 0 and x.dtype in (torch.float16, torch.bfloat16, torch.float32)):
        return _C.gemm.column_sum(x.reshape(-1, x.shape[-1]), out_dtype)
    # torch fallback: accumulate in at least fp32 (fp64 stays fp64: a double-precision gradcheck
    # of a FusedDense backward must not lose bits here)
    acc = torch.promote_types(x.dtype, torch.float32)
    return x.reshape(-1, x.shape[-1]).sum(0, dtype=acc).to(out_dtype)
