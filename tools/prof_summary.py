#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or ``kernel_stats.csv``).

The pyprof replacement's offline half (reference apex/pyprof/parse + prof): per-kernel calls,
total / average device time, share of GPU-busy time, plus the wall span of the trace, GPU busy
fraction and per-category totals (our native kernels vs MIOpen / hipBLASLt / torch elementwise).

Usage: python tools/prof_summary.py gpurun_out/prof_bench/bench_results.db [--top 40] [--md out.md]
"""
import argparse
import collections
import os
import re
import sqlite3
import sys

CATEGORIES = [
    ("apex_amd (native gfx950)", re.compile(r"apex_amd::")),
    ("batchnorm (MIOpen)", re.compile(r"BatchNorm", re.I)),
    ("RCCL", re.compile(r"nccl|rccl", re.I)),
    ("conv (MIOpen igemm / CK)", re.compile(r"igemm|naive_conv|conv|gridwise|ck::|ck16", re.I)),
    ("BLAS (hipBLASLt/rocBLAS/Tensile)", re.compile(r"Cijk_|Tensile|hipblaslt|rocblas", re.I)),
    ("torch elementwise/reduce", re.compile(r"at::native", re.I)),
]


def category(name):
    for cat, rx in CATEGORIES:
        if rx.search(name):
            return cat
    return "other"


def load_db(path, after=None):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    rows = [(n, int(s), int(e)) for n, s, e in rows]
    if after:
        rx = re.compile(after)
        idx = [i for i, (n, _, _) in enumerate(rows) if rx.search(n)]
        if idx:
            rows = rows[idx[-1] + 1:]
    return rows


def busy_time(intervals):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def short(name, n=110):
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= n else name[: n - 3] + "..."


def summarize(rows, top):
    agg = collections.defaultdict(lambda: [0, 0])
    cats = collections.defaultdict(int)
    for n, s, e in rows:
        agg[n][0] += 1
        agg[n][1] += e - s
        cats[category(n)] += e - s
    total = sum(v[1] for v in agg.values())
    span = (max(e for _, _, e in rows) - min(s for _, s, _ in rows)) if rows else 0
    busy = busy_time([(s, e) for _, s, e in rows])
    lines = []
    lines.append(f"dispatches: {len(rows)}  kernel-time sum: {total / 1e6:.3f} ms  GPU-busy: {busy / 1e6:.3f} ms  "
                 f"trace span: {span / 1e6:.3f} ms  busy/span: {100.0 * busy / max(span, 1):.1f}%")
    lines.append("")
    lines.append("| category | time (ms) | share |")
    lines.append("|---|---|---|")
    for cat, t in sorted(cats.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {cat} | {t / 1e6:.3f} | {100.0 * t / max(total, 1):.1f}% |")
    lines.append("")
    lines.append("| kernel | calls | total (ms) | avg (us) | share |")
    lines.append("|---|---|---|---|---|")
    for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"| `{short(n)}` | {cnt} | {t / 1e6:.3f} | {t / cnt / 1e3:.1f} | {100.0 * t / max(total, 1):.1f}% |")
    return "\n".join(lines)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    ap.add_argument("--title", default=None)
    ap.add_argument("--after", default=None, help="keep only dispatches after the last kernel matching this regex")
    ap.add_argument("--steps", type=int, default=None, help="report per-step times for this many steps")
    a = ap.parse_args(argv)
    rows = load_db(a.trace, a.after)
    text = summarize(rows, a.top)
    if a.steps:
        span = (max(e for _, _, e in rows) - min(s for _, s, _ in rows)) if rows else 0
        text = f"steps: {a.steps}  span per step: {span / 1e6 / a.steps:.3f} ms\n" + text
    if a.title:
        text = f"# {a.title}\n\nsource: `{os.path.basename(a.trace)}` (rocprofv3 --kernel-trace --stats)\n\n" + text
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
