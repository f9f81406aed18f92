#!/usr/bin/env python3
"""3x3 stride-1 forward / data gradient at the ResNet-50 bs-256 shapes: the halo-tile kernel
(csrc/conv/conv3x3_halo.hip) vs the r04 tap GEMM (fprop2, per-shape default config) vs MIOpen,
interleaved rounds in one process, random operands; JSON lines with median us and TFLOP/s."""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex  # noqa: F401,E402
from apex import _native  # noqa: E402
from apex.ops import conv as C  # noqa: E402

SHAPES = [(28, 128, 128), (14, 256, 256), (7, 512, 512), (56, 128, 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    ext = _native.require("conv").conv
    dev = torch.device("cuda")
    for h, cin, cout in SHAPES:
        n = args.batch if h != 56 else 64
        x = torch.randn(n, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        gy = torch.randn(n, cout, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        shift = torch.zeros(cout, device=dev)
        flop = 2.0 * n * h * h * cout * cin * 9

        def hfp_fwd():
            return C.conv_tap_forward(x, w, 1, 1, stats_shift=shift)

        def hfp_dgrad():
            return C.conv_tap_dgrad(gy, w, x.shape, 1, 1)

        def tap_fwd():
            ext.force_fprop_cfg(12 if cout % 256 == 0 else 11)
            try:
                return C.conv_tap_forward(x, w, 1, 1, stats_shift=shift)
            finally:
                ext.force_fprop_cfg(-1)

        def tap_dgrad():
            ext.force_fprop_cfg(12 if cin % 256 == 0 else 11)
            try:
                return C.conv_tap_dgrad(gy, w, x.shape, 1, 1)
            finally:
                ext.force_fprop_cfg(-1)

        def mi_fwd():
            return F.conv2d(x, w, None, 1, 1)

        def mi_dgrad():
            return torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [True, False, False])[0]

        engines = {"hfp_fwd": hfp_fwd, "tap_fwd": tap_fwd, "miopen_fwd": mi_fwd,
                   "hfp_dgrad": hfp_dgrad, "tap_dgrad": tap_dgrad, "miopen_dgrad": mi_dgrad}
        ref = mi_fwd().float()
        err = float((hfp_fwd()[0].float() - ref).abs().max()) / float(ref.abs().max())
        print(json.dumps({"check": f"{h}x{h}x{cin}->{cout}", "hfp_rel_err_vs_miopen": err}), flush=True)
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
        for name, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"shape": f"{h}x{h}x{cin}->{cout}", "n": n, "engine": name, "us_median": round(med, 1),
                              "us_min": round(min(ts), 1), "tflops": round(flop / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
