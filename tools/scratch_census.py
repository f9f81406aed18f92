#!/usr/bin/env python3
"""Register / scratch census of every kernel in a rocprofv3 --kernel-trace CSV: one line per
distinct kernel with its VGPR / AGPR / scratch bytes per lane, LDS, total time and calls —
private arrays the compiler put in scratch show up as Scratch_Size > 0.
Usage: python tools/scratch_census.py <kernel_trace.csv> [--all]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    show_all = "--all" in sys.argv
    agg = {}
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        k = (n, r.get("Scratch_Size", "0"), r.get("VGPR_Count", "?"), r.get("Accum_VGPR_Count", "?"))
        d = agg.setdefault(k, [0, 0.0])
        d[0] += 1
        d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print("| kernel | scratch B/lane | VGPR | AGPR | calls | total us |")
    print("|---|---|---|---|---|---|")
    for (n, sc, vg, ag), (c, us) in rows:
        if show_all or int(sc or 0) > 0:
            print(f"| `{n[:110]}` | {sc} | {vg} | {ag} | {c} | {us:.0f} |")


if __name__ == "__main__":
    main()
