#!/usr/bin/env python3
"""The ResNet-50 1x1 convolutions that run on the library route (stages 3-4 and the wide
stage-2 ones, bs 256): torch.matmul / addmm (hipBLASLt, the heuristic's first answer) against the
wrapper's per-shape top-8 timed plan (lt_gemm.mm), forward (x W^T) and data gradient (g W).
One JSON line per (shape, op).  Run on the GPU box: python tools/conv1x1_lt_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

SHAPES = [  # (M = n h w, Cin, Cout)
    (200704, 512, 256), (50176, 256, 1024), (50176, 1024, 256), (50176, 1024, 512),
    (12544, 512, 2048), (12544, 2048, 512), (50176, 512, 1024), (12544, 1024, 2048),
]


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import apex  # noqa: F401
    from apex import _native

    lt = _native.require("lt_gemm").lt_gemm
    dt = torch.bfloat16
    for m, cin, cout in SHAPES:
        x = torch.randn(m, cin, device="cuda", dtype=dt)
        w = torch.randn(cout, cin, device="cuda", dtype=dt) * 0.05
        g = torch.randn(m, cout, device="cuda", dtype=dt)
        r = {"m": m, "cin": cin, "cout": cout}
        r["fwd_torch_us"] = round(timeit(lambda: torch.matmul(x, w.t())), 1)
        r["fwd_lt_us"] = round(timeit(lambda: lt.mm(x, w, False, True)), 1)
        r["dgrad_torch_us"] = round(timeit(lambda: torch.matmul(g, w)), 1)
        r["dgrad_lt_us"] = round(timeit(lambda: lt.mm(g, w, False, False)), 1)
        ref = torch.matmul(x, w.t()).float()
        r["fwd_rel"] = float((lt.mm(x, w, False, True)[0].float() - ref).norm() / ref.norm())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
