#!/usr/bin/env python3
"""Per-shape timing of the BN-fused 1x1 convolution kernel (csrc/conv/conv1x1_bn.hip) against
MIOpen (F.conv2d / aten.convolution_backward) and hipBLASLt (torch.matmul on the NHWC views) for
every 1x1 stride-1 convolution of ResNet-50 at bs 256, bf16.  Forward arms: plain, + BN
statistics epilogue, + BN-apply/ReLU prologue and statistics; data-gradient arm: the
transposed-weight form.  Reports us and the HBM rate over the compulsory bytes (read A once,
write Y once).  One JSON line per (op, shape); one process, interleaved rounds.
Usage: python tools/bn1x1_bench.py [--rounds 3] [--iters 20] [--out FILE]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex  # noqa: E402

N = 256
ONE = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
       (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    ext = apex._native.require("conv").conv
    dev = torch.device("cuda")
    cl = torch.channels_last
    lines = []
    for h, cin, cout in ONE:
        m = N * h * h
        x = torch.randn(N, cin, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        gy = torch.randn(N, cout, h, h, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        w = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).to(memory_format=cl)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
        w2 = w.view(cout, cin)
        pcoef = torch.cat([torch.ones(cin, device=dev), torch.zeros(cin, device=dev)])
        shift = torch.zeros(cout, device=dev)
        ok_f = cin in (64, 128, 256, 512)
        ok_d = cout in (64, 128, 256, 512)
        arms = {"fwd": {"miopen": lambda: F.conv2d(x, w), "hipblaslt": lambda: torch.matmul(x2, w2.t())},
                "dgrad": {"miopen": lambda: torch.ops.aten.convolution_backward(
                    gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]),
                    "hipblaslt": lambda: torch.matmul(gy2, w2)}}
        if ok_f:
            arms["fwd"]["native"] = lambda: ext.bn1x1(x2, w2, False)
            arms["fwd"]["native_stats"] = lambda: ext.bn1x1(x2, w2, False, None, shift, True)
            arms["fwd"]["native_pro_stats"] = lambda: ext.bn1x1(x2, w2, False, pcoef, shift, True)
        if ok_d:
            arms["dgrad"]["native"] = lambda: ext.bn1x1(gy2, w2, True)
        arms["wgrad"] = {"miopen": lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]),
            "native": lambda: ext.wgrad1x1(gy2, x2),
            "native_pro": lambda: ext.wgrad1x1(gy2, x2, pcoef)}
        if os.environ.get("BN1X1_BENCH_ONLY_WGRAD"):
            arms = {"wgrad": arms["wgrad"]}
        res = {op: {k: [] for k in a} for op, a in arms.items()}
        for _ in range(args.rounds):
            for op, a in arms.items():
                for k, fn in a.items():
                    res[op][k].append(timeit(fn, args.iters))
        for op, a in res.items():
            mb = m * (cin + cout) * 2 / 1e6
            rec = {"op": op + "_1x1", "h": h, "cin": cin, "cout": cout, "m": m, "compulsory_MB": round(mb, 1)}
            for k, v in a.items():
                rec[k + "_us"] = round(min(v), 1)
                rec[k + "_TBps"] = round(mb / min(v), 2)  # MB / us = TB/s
            lines.append(rec)
            print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
