#!/usr/bin/env python3
"""3x3 stride-1 weight gradient at the ResNet-50 bs-256 shapes: the halo-tile kernel
(csrc/conv/conv3x3_wgrad.hip) vs the r04 native per-tap kernel (wgrad2 128 x 64) vs MIOpen
(aten.convolution_backward), interleaved rounds in one process (cdna_hip_programming.md rule 24),
random operands.  One JSON line per (shape, engine) with the median time and TFLOP/s."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import apex  # noqa: F401
from apex import _native
from apex.ops import conv as C

SHAPES = [(56, 64, 64), (28, 128, 128), (14, 256, 256), (7, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    ext = _native.require("conv").conv
    dev = torch.device("cuda")
    for h, cin, cout in SHAPES:
        n = args.batch
        x = torch.randn(n, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gy = torch.randn(n, cout, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.empty(cout, cin, 3, 3, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * n * h * h * cout * cin * 9

        def halo():
            ext.force_wgrad_variant(ext.WGRAD_HALO)
            return C.conv_tap_wgrad(gy, x, w.shape, 1, 1, torch.bfloat16)

        def tap():
            ext.force_wgrad_variant(3)
            return C.conv_tap_wgrad(gy, x, w.shape, 1, 1, torch.bfloat16)

        def miopen():
            return torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [False, True, False])[1]

        engines = {"halo": halo, "wgrad2": tap, "miopen": miopen}
        if args.check:
            ref = miopen().float()
            for name in ("halo", "wgrad2"):
                got = engines[name]().float()
                err = float((got - ref).abs().max()) / max(1e-6, float(ref.abs().max()))
                print(json.dumps({"check": name, "h": h, "c": cin, "rel_err_vs_miopen": err}), flush=True)
        times = {k: [] for k in engines}
        for fn in engines.values():
            fn()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for name, fn in engines.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    fn()
                e.record()
                e.synchronize()
                times[name].append(s.elapsed_time(e) * 1000.0 / args.iters)
        ext.force_wgrad_variant(-1)
        for name, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": f"{h}x{h}x{cin}->{cout}", "n": n, "engine": name, "us_median": round(med, 1),
                              "us_min": round(min(ts), 1), "tflops": round(flop / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
