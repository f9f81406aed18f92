"""Second stage of pyprof (reference apex/pyprof/prof/prof.py:171-256): read the parse stage's
per-kernel records, price each with its op model (FLOPs, bytes, parameters, MFMA use) and print
a columned table, CSV, or an aggregate summary.

``python -m apex.pyprof.prof [-c idx,dir,op,kernel,params,sil,tc,flops,bytes] [--csv | -w N]
[--summary op] parsed.txt``"""
import ast

from .base import param_string
from .ops import model
from .output import render, summary
from .usage import parse_args


def annotate(rec):
    """Attach flops / bytes / params / tc / achieved rates to one parsed record (in place)."""
    if rec.get("op"):
        m = model(rec)
        rec["flops"], rec["bytes"] = m.flops(), m.bytes()
        rec["params"], rec["tc"], rec["kind"] = param_string(m.params()), m.tc(), m.kind
    else:  # kernel outside any annotated op
        rec["flops"], rec["bytes"], rec["params"], rec["tc"], rec["kind"] = 0, 0, "", "-", "-"
    dur = max(1, int(rec.get("kDuration", 0) or 0))
    rec["tflops"] = "{:.1f}".format(rec["flops"] / dur / 1e3) if rec["flops"] else "-"
    rec["gbps"] = "{:.0f}".format(rec["bytes"] / dur) if rec["bytes"] else "-"
    rec["layerStr"] = "/".join(rec.get("layer", []) or [])
    rec["traceStr"] = ";".join((rec.get("trace", []) or [])[-1:])
    rec["gridStr"] = ",".join(str(x) for x in rec.get("grid", ()))
    rec["blockStr"] = ",".join(str(x) for x in rec.get("block", ()))
    return rec


def foo(mod, op, d):
    """The op model pricing ``op`` of module ``mod`` for the kernel record ``d`` (a ``Data``);
    the reference's dispatch entry point (apex/pyprof/prof/prof.py:27-169)."""
    return model(d.record(mod, op))


def attribute_to_main_kernel(records):
    """An op launches several kernels (fills, transposes, the GEMM, a reduction); its modelled
    FLOPs / bytes are charged once, to the longest kernel of the op instance (same thread,
    seqId and direction), so per-kernel rates and aggregates are not multiplied."""
    groups = {}
    for r in records:
        if r.get("op") and r.get("seqId", -1) >= 0:
            groups.setdefault((r.get("tid"), r.get("seqId"), r.get("dir")), []).append(r)
    for rs in groups.values():
        main = max(rs, key=lambda r: int(r.get("kDuration", 0) or 0))
        for r in rs:
            if r is not main:
                r["flops"] = r["bytes"] = 0
                r["tflops"] = r["gbps"] = "-"
    return records


def read_records(f):
    for line in f:
        line = line.strip()
        if line.startswith("{"):
            yield ast.literal_eval(line)


def main(argv=None):
    a = parse_args(argv)
    recs = attribute_to_main_kernel([annotate(r) for r in read_records(a.file)])
    if a.summary:
        print(summary(recs, a.summary, a.top))
    else:
        print(render(recs, a.c, a.csv, a.w))
    return 0
