#!/usr/bin/env python3
"""Per-shape A/B of the ResNet-50 (bs 256, bf16, channels_last) convolution backward routes on
one box, one process, interleaved rounds:

* 1x1 stride-1 weight gradient  dW = gy^T x over the [pixels, C] views:
  MIOpen (aten.convolution_backward), hipBLASLt (torch.matmul), native split-K GEMM
* 1x1 stride-1 data gradient   dx = gy W:  MIOpen, hipBLASLt, native
* 1x1 stride-1 forward          y = x W^T:  MIOpen, hipBLASLt, native
* 3x3 weight gradient: MIOpen vs the native implicit-GEMM wgrad

MIOpen's time includes its helper launches (output zero-fill, fp32->bf16 cast) because the
timing brackets the whole call.  One JSON line per (op, shape).
Usage: python tools/conv_bwd_ab.py [--rounds 3] [--iters 10]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex  # noqa: E402
from apex.ops import conv as conv_ops  # noqa: E402

N = 256
# (H, Cin, Cout) of every 1x1 stride-1 conv of ResNet-50 (dedup)
ONE = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
       (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048), (7, 2048, 512)]
# (H_in, C, K, stride) of the 3x3 convs
THREE = [(56, 64, 64, 1), (56, 128, 128, 2), (28, 128, 128, 1), (28, 256, 256, 2), (14, 256, 256, 1),
         (14, 512, 512, 2), (7, 512, 512, 1)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    g = apex._native.require("conv1x1").gemm
    ext = apex._native.require("conv").conv
    dev = torch.device("cuda")
    cl = torch.channels_last
    for h, cin, cout in ([] if os.environ.get("CONV_AB_ONLY_3X3") else ONE):
        x = torch.randn(N, cin, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        gy = torch.randn(N, cout, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        w = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).to(memory_format=cl)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
        w2 = w.view(cout, cin)
        arms = {
            "wgrad": {
                "miopen": lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False]),
                "hipblaslt": lambda: torch.matmul(gy2.t(), x2),
                "native": lambda: g.linear_wgrad(gy2, x2),
            },
            "dgrad": {
                "miopen": lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                      [0, 0], 1, [True, False, False]),
                "hipblaslt": lambda: torch.matmul(gy2, w2),
                "native": lambda: g.linear_dgrad(gy2, w2, g.EPI_NONE, None),
            },
            "fwd": {
                "miopen": lambda: F.conv2d(x, w),
                "hipblaslt": lambda: torch.matmul(x2, w2.t()),
                "native": lambda: g.linear(x2, w2, None, g.EPI_NONE, False),
            },
        }
        for op, fns in arms.items():
            res = {k: [] for k in fns}
            for _ in range(args.rounds):
                for k, fn in fns.items():
                    res[k].append(timeit(fn, args.iters))
            line = {"op": op + "_1x1", "h": h, "cin": cin, "cout": cout, "m": N * h * h}
            line.update({k + "_us": round(min(v), 1) for k, v in res.items()})
            best = min(fns, key=lambda k: min(res[k]))
            line["best"] = best
            print(json.dumps(line), flush=True)
        del x, gy, w, x2, gy2
    for h, c, k, st in THREE:
        x = torch.randn(N, c, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        ho = h // st
        gy = torch.randn(N, k, ho, ho, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        w = (torch.randn(k, c, 3, 3, device=dev, dtype=torch.bfloat16) * 0.05).to(memory_format=cl)
        fns = {
            "miopen": lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [st, st], [1, 1], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]),
            "native_gather": lambda: ext.wgrad3x3(gy.permute(0, 2, 3, 1), x.permute(0, 2, 3, 1), st),
        }

        def variant(v):
            def f():
                ext.force_wgrad_variant(v)
                try:
                    return conv_ops.conv_tap_wgrad(gy, x, w.shape, st, 1, w.dtype)
                finally:
                    ext.force_wgrad_variant(-1)
            return f

        for v in range(5):  # 0 wgrad_kernel, 1-4 wgrad2_kernel tiles (launch_plan.h conv_wgrad)
            fns[f"native_v{v}"] = variant(v)
        res = {kk: [] for kk in fns}
        for _ in range(args.rounds):
            for kk, fn in fns.items():
                res[kk].append(timeit(fn, args.iters))
        line = {"op": "wgrad_3x3", "h": h, "c": c, "k": k, "stride": st}
        line.update({kk + "_us": round(min(v), 1) for kk, v in res.items()})
        line["best"] = min(fns, key=lambda kk: min(res[kk]))
        print(json.dumps(line), flush=True)
        del x, gy, w


if __name__ == "__main__":
    main()
