#!/usr/bin/env python3
"""Idle gaps of a rocprofv3 kernel trace: total device idle time between consecutive kernels,
attributed to the kernel that ran BEFORE each gap (where the host fell behind), plus a
histogram.  Usage: python tools/prof_gaps.py results.db [--after spin_kernel] [--min-us 5]"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import load_db, short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--after", default=None)
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    rows = load_db(a.trace, a.after)
    end = None
    prev = None
    by_prev = collections.defaultdict(lambda: [0, 0.0])
    hist = collections.Counter()
    total = 0.0
    for n, s, e in rows:
        if end is not None and s > end:
            gap = (s - end) / 1e3
            total += gap
            if gap >= a.min_us:
                by_prev[prev][0] += 1
                by_prev[prev][1] += gap
            hist[min(int(gap // 10) * 10, 200)] += 1
        if end is None or e > end:
            end = e
            prev = n
    print(f"idle total {total / 1e3:.3f} ms over {len(rows)} dispatches")
    print("gap-us-bucket count: " + ", ".join(f"{k}:{v}" for k, v in sorted(hist.items())))
    print("| kernel before the gap | gaps >= %.0f us | idle (ms) |" % a.min_us)
    print("|---|---|---|")
    for n, (c, t) in sorted(by_prev.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"| `{short(n, 100)}` | {c} | {t / 1e3:.3f} |")


if __name__ == "__main__":
    main()
