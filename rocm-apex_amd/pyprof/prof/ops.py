"""Op -> model registry (reference apex/pyprof/prof/prof.py:27-169 dispatch chain).

Every model module exports ``OPS`` (torch / functional / Tensor op names) and ``MODULES``
(``nn.Module`` class names whose ``forward`` marker is priced directly).  Unknown ops fall back
to ``Foo``: no FLOPs, bytes = the tensors in its marker."""
from . import blas, conv, data_movement, normalization, optim, pointwise, reduction
from .base import OpModel, param_string

_FAMILIES = (pointwise, data_movement, reduction, normalization, conv, blas, optim)
OPS, MODULES = {}, {}
for _m in _FAMILIES:  # later families win on name clashes (GEMM / conv over generic names)
    OPS.update(_m.OPS)
    MODULES.update(_m.MODULES)


class Foo(OpModel):
    kind = "other"


def model(rec):
    op, mod = rec.get("op", ""), rec.get("mod", "")
    if op == "forward" and mod in MODULES:
        return MODULES[mod](rec)
    cls = OPS.get(op)
    if cls is None and op.endswith("_"):
        cls = OPS.get(op[:-1])
    return (cls or Foo)(rec)


def model_for(rec):
    """(flops, bytes, params-string) of one parsed record (kept for callers of the round-1 API)."""
    if not rec.get("op"):
        return 0, 0, ""
    m = model(rec)
    return m.flops(), m.bytes(), param_string(m.params())
