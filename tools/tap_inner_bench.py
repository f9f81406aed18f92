#!/usr/bin/env python3
"""The tap-GEMM 3x3 forward / data gradient (csrc/conv/conv_igemm.hip) at the ResNet-50 stage-2/3/4
shapes: plain, with the BN-statistics epilogue (as the node runs it), and back-to-back after a
streaming pass that evicts the L2 / MALL (as in the step, where the producer wrote other tensors
in between) — to place the gap between the standalone sweep (profiles/r05/conv_cfg_sweep_r05j.jsonl)
and the in-step times.  One JSON line per (shape, variant)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import apex  # noqa: E402,F401
from apex.ops import conv as C  # noqa: E402


def timeit(fn, iters=20, warmup=3, flush=None):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(iters):
        if flush is not None:
            flush()
        s.record()
        fn()
        e.record()
        e.synchronize()
        tot += s.elapsed_time(e)
    return tot / iters * 1e3


def main():
    ext = C._conv_ext()
    big = torch.empty(512 * 1024 * 1024 // 2, device="cuda", dtype=torch.bfloat16)
    big2 = torch.empty_like(big)
    flush = lambda: big2.copy_(big)  # noqa: E731  1 GB moved: evicts L2 and the 256 MB MALL
    for c, h in [(128, 28), (256, 14), (512, 7)]:
        x = torch.randn(256, c, h, h, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda", dtype=torch.bfloat16) * 0.05).to(memory_format=torch.channels_last)
        gy = torch.randn(256, c, h, h, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        shift = torch.zeros(c, device="cuda")
        rows = {
            "fwd": lambda: C.conv_tap_forward(x, w, 1, 1),
            "fwd_stats": lambda: C.conv_tap_forward(x, w, 1, 1, stats_shift=shift),
            "dgrad": lambda: C.conv_tap_dgrad(gy, w, x.shape, 1, 1),
        }
        for name, fn in rows.items():
            warm = timeit(fn)
            cold = timeit(fn, flush=flush)
            print(json.dumps({"c": c, "h": h, "op": name, "warm_us": round(warm, 1), "cold_us": round(cold, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
