"""Kernel / marker correlation for rocprofv3 traces (reference apex/pyprof/parse/parse.py,
nvvp.py, db.py, kernel.py, which read nvprof's SQLite output).

Input: a rocprofv3 output directory or file —
  * rocpd SQLite (``*_results.db``): the ``kernels`` view (and marker / region views if the run
    used ``--marker-trace``),
  * CSV (``--output-format csv``): ``*kernel_trace.csv`` plus, when present,
    ``*marker_api_trace.csv`` and ``*hip_api_trace.csv``.
Each kernel is attributed to the innermost marker range (``apex.pyprof.nvtx`` op markers)
enclosing the HOST call that launched it: kernel -> launching HIP API call via the correlation
id -> thread + host timestamp -> marker stack on that thread.  Without a HIP API trace the
kernel's own start time is used (good enough for synchronous / serialized runs).

Output (``python -m apex.pyprof.parse <trace>``): one python-literal dict per kernel per line,
the format the reference's parse stage emits and ``apex.pyprof.prof`` consumes.
"""
import ast
import bisect
import csv
import glob
import os
import sqlite3
import sys


def _find(path, pattern):
    if os.path.isfile(path):
        return [path] if pattern in os.path.basename(path) else []
    return sorted(glob.glob(os.path.join(path, "**", "*" + pattern), recursive=True))


def _col(header, *cands):
    low = [h.lower() for h in header]
    for c in cands:
        c = c.lower()
        for i, h in enumerate(low):
            if h == c:
                return i
    for c in cands:
        c = c.lower()
        for i, h in enumerate(low):
            if c in h:
                return i
    return None


def _int(v, default=0):
    """rocprofv3 writes some ids as text ("Agent 2"): keep the trailing integer."""
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError:
        digits = "".join(ch for ch in str(v).split()[-1] if ch.isdigit())
        return int(digits) if digits else default


def _read_csv(path):
    with open(path, newline="") as f:
        r = csv.reader(f)
        header = next(r)
        return header, list(r)


def load_csv(path):
    kernels, markers, api = [], [], {}
    for kpath in _find(path, "kernel_trace.csv"):
        h, rows = _read_csv(kpath)
        ci = {k: _col(h, *v) for k, v in {
            "name": ("Kernel_Name", "KernelName", "name"), "start": ("Start_Timestamp", "start"),
            "end": ("End_Timestamp", "end"), "corr": ("Correlation_Id",), "tid": ("Thread_Id",),
            "gx": ("Grid_Size_X", "Grid_Size"), "gy": ("Grid_Size_Y",), "gz": ("Grid_Size_Z",),
            "bx": ("Workgroup_Size_X", "Workgroup_Size"), "by": ("Workgroup_Size_Y",), "bz": ("Workgroup_Size_Z",),
            "queue": ("Queue_Id", "Stream_Id"), "agent": ("Agent_Id", "Device_Id")}.items()}
        for row in rows:
            g = lambda k, d=None: row[ci[k]] if ci[k] is not None and ci[k] < len(row) else d  # noqa: E731
            kernels.append({"name": g("name"), "start": _int(g("start")), "end": _int(g("end")),
                            "corr": _int(g("corr"), -1), "tid": _int(g("tid"), -1),
                            "grid": tuple(_int(g(k), 1) for k in ("gx", "gy", "gz")),
                            "block": tuple(_int(g(k), 1) for k in ("bx", "by", "bz")),
                            "stream": _int(g("queue")), "device": _int(g("agent"))})
    for mpath in _find(path, "marker_api_trace.csv"):
        h, rows = _read_csv(mpath)
        fi, si, ei, ti = (_col(h, "Function", "Message"), _col(h, "Start_Timestamp"), _col(h, "End_Timestamp"),
                          _col(h, "Thread_Id"))
        for row in rows:
            markers.append((_int(row[ti], -1) if ti is not None else -1, _int(row[si]), _int(row[ei]), row[fi]))
    for apath in _find(path, "hip_api_trace.csv"):
        h, rows = _read_csv(apath)
        ci, si, ti = _col(h, "Correlation_Id"), _col(h, "Start_Timestamp"), _col(h, "Thread_Id")
        for row in rows:
            api[_int(row[ci])] = (_int(row[ti], -1) if ti is not None else -1, _int(row[si]))
    return kernels, markers, api


def load_db(path):
    dbs = _find(path, ".db")
    kernels, markers = [], []
    for db in dbs:
        c = sqlite3.connect(db)
        views = {r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")}
        if "kernels" in views:
            cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
            want = [x for x in ("name", "start", "end", "grid_size_x", "grid_size_y", "grid_size_z",
                                "workgroup_size_x", "workgroup_size_y", "workgroup_size_z", "stream_id",
                                "queue_id", "tid", "correlation_id") if x in cols]
            for row in c.execute("select {} from kernels order by start".format(",".join(want))):
                d = dict(zip(want, row))
                kernels.append({"name": d["name"], "start": int(d["start"]), "end": int(d["end"]),
                                "corr": int(d.get("correlation_id", -1) or -1), "tid": int(d.get("tid", -1) or -1),
                                "grid": tuple(int(d.get(k, 1) or 1) for k in ("grid_size_x", "grid_size_y",
                                                                              "grid_size_z")),
                                "block": tuple(int(d.get(k, 1) or 1) for k in ("workgroup_size_x",
                                                                               "workgroup_size_y",
                                                                               "workgroup_size_z")),
                                "stream": int(d.get("stream_id", d.get("queue_id", 0)) or 0), "device": 0})
        for v in ("regions", "markers"):
            if v in views:
                cols = [r[1] for r in c.execute("pragma table_info({})".format(v))]
                if {"name", "start", "end"} <= set(cols):
                    tid = "tid" if "tid" in cols else "-1"
                    for name, s, e, t in c.execute("select name, start, end, {} from {}".format(tid, v)):
                        markers.append((int(t), int(s), int(e), name))
                break
    return kernels, markers, {}


def attach_markers(kernels, markers, api):
    """kernel -> innermost marker range containing its launch time (same thread when known)."""
    by_tid = {}
    for tid, s, e, text in markers:
        by_tid.setdefault(tid, []).append((s, e, text))
    for v in by_tid.values():
        v.sort()
    any_tid = sorted(m for v in by_tid.values() for m in v)
    for k in kernels:
        tid, t = k["tid"], k["start"]
        if k["corr"] in api:
            tid, t = api[k["corr"]]
        ranges = by_tid.get(tid, any_tid)
        starts = [r[0] for r in ranges]
        i = bisect.bisect_right(starts, t)
        enclosing = [r for r in ranges[max(0, i - 256):i] if r[0] <= t <= r[1]]
        k["markers"] = [r[2] for r in enclosing]
        k["ranges"] = enclosing
    return split_markers(kernels)


def _is_layer(text):
    return isinstance(text, str) and text.startswith("layer:")


def split_markers(kernels):
    """Per kernel: the innermost op marker (ignoring ``layer:`` annotations), the enclosing
    layer path, and the sub-index of the kernel among those launched inside the same op range."""
    counters = {}
    for k in kernels:
        ranges = k.get("ranges", [])
        ops = [r for r in ranges if not _is_layer(r[2])]
        layers = sorted((r for r in ranges if _is_layer(r[2])), key=lambda r: r[0])
        k["layer"] = [r[2][len("layer:"):] for r in layers]
        if ops:
            inner = min(ops, key=lambda r: r[1] - r[0])
            k["marker"] = inner[2]
            key = (k.get("tid"), inner[0], inner[2])
            k["sub"] = counters.get(key, 0)
            counters[key] = k["sub"] + 1
        else:
            k["marker"], k["sub"] = None, 0
    return kernels


def decode_marker(text):
    """The apex.pyprof.nvtx payload (python-literal dict) or {} for foreign markers."""
    if not text:
        return {}
    try:
        d = ast.literal_eval(text)
        return d if isinstance(d, dict) else {}
    except (ValueError, SyntaxError):
        return {"op": text}


def parse(path):
    kernels, markers, api = ([], [], {})
    if _find(path, ".db"):
        kernels, markers, api = load_db(path)
    if not kernels:
        kernels, markers, api = load_csv(path)
    kernels.sort(key=lambda k: k["start"])
    attach_markers(kernels, markers, api)
    out = []
    for i, k in enumerate(kernels):
        m = decode_marker(k["marker"])
        out.append({"index": i, "kName": k["name"], "kStartTime": k["start"], "kEndTime": k["end"],
                    "kDuration": k["end"] - k["start"], "grid": k["grid"], "block": k["block"],
                    "device": k["device"], "stream": k["stream"], "tid": k.get("tid", -1),
                    "mod": m.get("mod", ""), "op": m.get("op", ""), "dir": m.get("dir", "fprop" if m else ""),
                    "seqId": m.get("seqId", -1), "sub": k.get("sub", 0), "layer": m.get("layer") or k.get("layer", []),
                    "args": m.get("args", []), "strRepr": m.get("strRepr", ""),
                    "trace": m.get("traceMarker", []), "marker": k["marker"]})
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print("usage: python -m apex.pyprof.parse <rocprofv3 output dir | results.db | kernel_trace.csv>")
        return 2
    for rec in parse(argv[0]):
        print(rec)
    return 0
