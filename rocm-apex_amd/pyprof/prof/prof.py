"""Second stage of pyprof (reference apex/pyprof/prof/prof.py + output.py): read the parse
stage's per-kernel records, attach FLOP / byte estimates from the op models and print a
columned table or CSV.

``python -m apex.pyprof.prof [-c idx,op,kernel,sil,flops,bytes] [--csv] [-w 160] parsed.txt``
(``parsed.txt`` = the output of ``python -m apex.pyprof.parse``; ``-`` reads stdin)."""
import argparse
import ast
import sys

from .ops import model_for

COLUMNS = {
    "idx": ("Idx", "index", 6), "mod": ("Module", "mod", 14), "op": ("Op", "op", 18),
    "kernel": ("Kernel", "kName", 0), "params": ("Params", "params", 0), "sil": ("Sil(ns)", "kDuration", 10),
    "grid": ("Grid", "grid", 14), "block": ("Block", "block", 12), "stream": ("Stream", "stream", 6),
    "device": ("Device", "device", 6), "flops": ("FLOPs", "flops", 14), "bytes": ("Bytes", "bytes", 14),
    "tflops": ("TFLOP/s", "tflops", 9), "gbps": ("GB/s", "gbps", 9),
}


def annotate(rec):
    flops, nbytes, params = model_for(rec)
    rec["flops"], rec["bytes"], rec["params"] = flops, nbytes, params
    dur = max(1, int(rec.get("kDuration", 0)))
    rec["tflops"] = "{:.1f}".format(flops / dur / 1e3) if flops else "-"
    rec["gbps"] = "{:.0f}".format(nbytes / dur) if nbytes else "-"
    return rec


def read_records(f):
    for line in f:
        line = line.strip()
        if line.startswith("{"):
            yield ast.literal_eval(line)


def render(records, cols, csv=False, width=0):
    out = []
    if csv:
        out.append(",".join(COLUMNS[c][0] for c in cols))
        for r in records:
            out.append(",".join('"{}"'.format(r.get(COLUMNS[c][1], "")) for c in cols))
        return "\n".join(out)
    fixed = sum(COLUMNS[c][2] for c in cols)
    flex = [c for c in cols if COLUMNS[c][2] == 0]
    fw = max(20, (width - fixed) // max(1, len(flex))) if width else 60
    widths = [COLUMNS[c][2] or fw for c in cols]
    out.append(" ".join(COLUMNS[c][0].ljust(w) for c, w in zip(cols, widths)))
    for r in records:
        out.append(" ".join(str(r.get(COLUMNS[c][1], ""))[:w].ljust(w) for c, w in zip(cols, widths)))
    return "\n".join(out)


def main(argv=None):
    ap = argparse.ArgumentParser(description="per-kernel FLOP / byte report from apex.pyprof.parse output")
    ap.add_argument("file", nargs="?", default="-")
    ap.add_argument("-c", default="idx,mod,op,kernel,sil,flops,bytes,tflops")
    ap.add_argument("--csv", action="store_true")
    ap.add_argument("-w", type=int, default=180)
    a = ap.parse_args(argv)
    f = sys.stdin if a.file == "-" else open(a.file)
    recs = [annotate(r) for r in read_records(f)]
    print(render(recs, a.c.split(","), a.csv, a.w))
    return 0
