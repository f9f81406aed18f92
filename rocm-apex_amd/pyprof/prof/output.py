"""Columned / CSV rendering of the annotated kernel records (reference
apex/pyprof/prof/output.py)."""

# column -> (header, record key, fixed width; 0 = share the remaining width)
COLUMNS = {
    "idx": ("Idx", "index", 6), "seq": ("SeqId", "seqId", 7), "tid": ("Tid", "tid", 9),
    "layer": ("Layer", "layerStr", 0), "trace": ("Trace", "traceStr", 0), "dir": ("Direction", "dir", 9),
    "sub": ("Sub", "sub", 4), "mod": ("Module", "mod", 16), "op": ("Op", "op", 18), "kernel": ("Kernel", "kName", 0),
    "params": ("Params", "params", 0), "sil": ("Sil(ns)", "kDuration", 10), "tc": ("TC", "tc", 3),
    "device": ("Device", "device", 6), "stream": ("Stream", "stream", 6), "grid": ("Grid", "gridStr", 14),
    "block": ("Block", "blockStr", 12), "flops": ("FLOPs", "flops", 14), "bytes": ("Bytes", "bytes", 14),
    "tflops": ("TFLOP/s", "tflops", 9), "gbps": ("GB/s", "gbps", 9), "kind": ("Kind", "kind", 13),
}
DEFAULT = "idx,dir,sub,mod,op,kernel,params,sil"


def _cell(rec, key):
    v = rec.get(key, "")
    return "" if v is None else str(v)


def render(records, cols, csv=False, width=0):
    out = []
    if csv:
        out.append(",".join(COLUMNS[c][0] for c in cols))
        for r in records:
            out.append(",".join('"{}"'.format(_cell(r, COLUMNS[c][1]).replace('"', "'")) for c in cols))
        return "\n".join(out)
    fixed = sum(COLUMNS[c][2] for c in cols)
    flex = [c for c in cols if COLUMNS[c][2] == 0]
    fw = max(20, (width - fixed - len(cols)) // max(1, len(flex))) if width else 60
    widths = [COLUMNS[c][2] or fw for c in cols]
    out.append(" ".join(COLUMNS[c][0].ljust(w) for c, w in zip(cols, widths)))
    for r in records:
        out.append(" ".join(_cell(r, COLUMNS[c][1])[:w].ljust(w) for c, w in zip(cols, widths)).rstrip())
    return "\n".join(out)


def summary(records, by="op", top=25):
    """Aggregate silicon time / FLOPs / bytes per op (or per kernel / module / layer)."""
    agg = {}
    for r in records:
        key = (r.get("dir", ""), r.get(by, "") if by != "layer" else r.get("layerStr", ""))
        a = agg.setdefault(key, {"n": 0, "ns": 0, "flops": 0, "bytes": 0})
        a["n"] += 1
        a["ns"] += int(r.get("kDuration", 0))
        a["flops"] += int(r.get("flops", 0) or 0)
        a["bytes"] += int(r.get("bytes", 0) or 0)
    total = max(1, sum(a["ns"] for a in agg.values()))
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])[:top]
    lines = ["{:<6} {:<40} {:>7} {:>12} {:>6} {:>9} {:>9}".format("dir", by, "calls", "time(us)", "%", "TFLOP/s",
                                                                  "GB/s")]
    for (d, k), a in rows:
        ns = max(1, a["ns"])
        lines.append("{:<6} {:<40} {:>7} {:>12.1f} {:>6.1f} {:>9.1f} {:>9.0f}".format(
            d[:6], str(k)[:40], a["n"], a["ns"] / 1e3, 100.0 * a["ns"] / total, a["flops"] / ns / 1e3,
            a["bytes"] / ns))
    return "\n".join(lines)
