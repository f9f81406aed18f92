#!/usr/bin/env python3
"""One training step of a rocprofv3 kernel trace in dispatch order: kernel, grid, workgroup,
duration and the gap to the previous kernel's end.  The step's layer structure is fixed, so the
position of a dispatch names its layer (e.g. the 3x3 convs of stage 3 are the 6 fprop launches
between the stage-3 1x1s); the per-kernel totals of prof_summary.py cannot tell shapes apart.

Usage: python tools/prof_timeline.py results.db --after spin_kernel --steps 10 --step 5 [--md out.md]
(``--step`` picks which of the ``--steps`` steps after the last ``--after`` marker to print: the
dispatches are split into ``--steps`` equal slices.)"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after", default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--step", type=int, default=5)
    ap.add_argument("--md", default=None)
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
    want = ["name", "start", "end"]
    for k in ("grid_size_x", "grid_size", "grid_x"):
        if k in cols:
            want.append(k)
            break
    for k in ("workgroup_x", "workgroup_size_x", "workgroup_size"):
        if k in cols:
            want.append(k)
            break
    rows = c.execute(f"select {', '.join(want)} from kernels order by start").fetchall()
    if args.after:
        rx = re.compile(args.after)
        idx = [i for i, r in enumerate(rows) if rx.search(r[0])]
        if idx:
            rows = rows[idx[-1] + 1:]
    per = len(rows) // max(1, args.steps)
    step = rows[args.step * per:(args.step + 1) * per]
    out = [f"<!-- columns available: {cols} -->",
           f"dispatches in step {args.step}: {len(step)}  (total {len(rows)} over {args.steps} steps)", "",
           "| # | kernel | grid | wg | us | gap us |", "|---|---|---|---|---|---|"]
    prev_end = None
    tot = 0.0
    for i, r in enumerate(step):
        name, s, e = r[0], int(r[1]), int(r[2])
        grid = r[3] if len(r) > 3 else ""
        wg = r[4] if len(r) > 4 else ""
        us = (e - s) / 1e3
        tot += us
        gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:.1f}"
        prev_end = e
        nm = re.sub(r"\(.*", "", name)[:120]
        out.append(f"| {i} | `{nm}` | {grid} | {wg} | {us:.1f} | {gap} |")
    out.append("")
    out.append(f"kernel time in the step: {tot:.1f} us")
    text = "\n".join(out)
    if args.md:
        with open(args.md, "w") as f:
            f.write(text + "\n")
    print("\n".join(out[:8]))


if __name__ == "__main__":
    main()
