#!/usr/bin/env python3
"""Join rocprofv3 hardware-counter passes (tools/gpu_pmc.sh) into one per-kernel table.

Each pass directory holds a ``*counter_collection.csv`` (one row per dispatch x counter) and the
kernel-trace pass a ``*kernel_trace.csv``.  Per kernel (name truncated) we report mean duration
and the mean of every counter, plus derived metrics:
  MFMA % peak = SQ_INSTS_MFMA x FLOP per MFMA (32768 for v_mfma_f32_32x32x16, 16384 for the
  v_mfma_f32_16x16x32 of the g8p GEMM kernels)
                / duration / 2.5 PFLOP/s dense bf16 peak
  LDS conf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles per LDS-array cycle)
  HBM GB/s   = (FETCH_SIZE + WRITE_SIZE) KiB / duration  (FETCH_SIZE under-counts wide streams on
               gfx950 by up to 2x: cdna_hip_programming.md §7 — read as a lower bound)
Usage: python tools/pmc_summary.py gpurun_out/pmc [--md profiles/pmc_kernels.md]"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[:90]


def _grid(r):
    g = r.get("Grid_Size")
    if g:
        return int(g)
    try:
        return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    except (KeyError, ValueError):
        return 0


def load(d, by_grid=False):
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    durations = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            nm = short(r["Kernel_Name"]) + (f" @grid{_grid(r)}" if by_grid else "")
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), nm)
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (_, k), vals in per.items():
            for c, v in vals.items():
                counters[k][c].append(v)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            nm = short(r["Kernel_Name"]) + (f" @grid{_grid(r)}" if by_grid else "")
            durations[nm].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return counters, durations


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--md")
    ap.add_argument("--filter", default="apex_amd::")
    ap.add_argument("--by-grid", action="store_true", help="one row per (kernel, grid size): per-shape rows")
    a = ap.parse_args()
    counters, durations = load(a.dir, a.by_grid)
    rows = []
    for k in sorted(set(counters) | set(durations)):
        if not any(f in k for f in a.filter.split("|")):
            continue
        c = {n: sum(v) / len(v) for n, v in counters[k].items()}
        dur = sorted(durations.get(k, [0.0]))[len(durations.get(k, [0.0])) // 2]
        nm = c.get("SQ_INSTS_MFMA")
        flop = 16384 if "g8p::" in k else 32768
        util = 100.0 * nm * flop / (dur * 1e-6) / 2.5e15 if nm and dur else (0.0 if nm == 0 else None)
        lds = c.get("SQ_LDS_BANK_CONFLICT"), c.get("SQ_LDS_IDX_ACTIVE")
        conf = 100.0 * lds[0] / lds[1] if lds[0] is not None and lds[1] else None
        fetch, write = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        gbs = (fetch + write) * 1024 / (dur * 1e3) if fetch is not None and write is not None and dur else None
        rows.append((k, dur, util, conf, fetch, write, gbs, c))
    extra = any("SQ_WAVE_CYCLES" in r[7] for r in rows)
    lines = ["| kernel | us (median) | MFMA % of 2.5 PF peak | LDS bank-conflict cycles % | FETCH KiB | WRITE KiB | HBM GB/s (lower bound) | MFMA insts | VALU insts | waves |"
             + (" wait-any % of wave cycles | wait-inst-any % | wait-inst-LDS % | VALU/MFMA co-exec cycles |" if extra else ""),
             "|---|---|---|---|---|---|---|---|---|---|" + ("---|---|---|---|" if extra else "")]
    fmt = lambda v, f="{:.1f}": "-" if v is None else f.format(v)  # noqa: E731
    for k, dur, util, conf, fetch, write, gbs, c in rows:
        lines.append("| `{}` | {} | {} | {} | {} | {} | {} | {} | {} | {} |".format(
            k, fmt(dur), fmt(util), fmt(conf), fmt(fetch, "{:.0f}"), fmt(write, "{:.0f}"), fmt(gbs, "{:.0f}"),
            fmt(c.get("SQ_INSTS_MFMA"), "{:.0f}"), fmt(c.get("SQ_INSTS_VALU"), "{:.0f}"),
            fmt(c.get("SQ_WAVES"), "{:.0f}")) + ("" if not extra else " {} | {} | {} | {} |".format(
                *[fmt(100.0 * c[n] / c["SQ_WAVE_CYCLES"] if c.get(n) is not None and c.get("SQ_WAVE_CYCLES") else None)
                  for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS")],
                fmt(c.get("SQ_VALU_MFMA_COEXEC_CYCLES"), "{:.0f}"))))
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write("# Hardware counters of the native gfx950 kernels (1 x MI355X, rocprofv3 --pmc)\n\n")
            f.write("Source: `tools/gpu_pmc.sh` (one rocprofv3 pass per counter group over `tools/pmc_kernels.py`),"
                    " joined by `tools/pmc_summary.py`. Mean over 3 calls per kernel.\n\n")
            f.write(out + "\n")


if __name__ == "__main__":
    main()
