#!/usr/bin/env python3
"""Weight-gradient GEMM dW[N, K] = g[M, N]^T x[M, K] at the transformer shapes (M = 16384 tokens):
torch (``g.t().matmul(x)``, hipBLASLt through PyTorch), our hipBLASLt call with explicit layouts
(``lt_gemm.wgrad_bgrad``, no bias) and the native split-K MFMA kernel (``gemm.linear_wgrad``).
One process, interleaved rounds; one JSON line per shape.  Usage: python tools/wgrad_shapes_ab.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex  # noqa: E402

SHAPES = [(16384, 3072, 1024), (16384, 1024, 1024), (16384, 4096, 1024), (16384, 1024, 4096),
          (8192, 1024, 1024), (32768, 1024, 4096)]


def timeit(fn, iters=10):
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
    g = apex._native.require("gemm").gemm
    lt = apex._native.submodule("lt_gemm")
    for m, n, k in SHAPES:
        go = torch.randn(m, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        ref = go.float().t() @ x.float()
        arms = {"torch": lambda: go.t().matmul(x), "native": lambda: g.linear_wgrad(go, x)}
        if lt is not None:
            arms["lt"] = lambda: lt.wgrad_bgrad(go, x, False)[0]
        res = {a: [] for a in arms}
        for _ in range(3):
            for a, fn in arms.items():
                res[a].append(timeit(fn))
        line = {"m": m, "n": n, "k": k}
        flop = 2.0 * m * n * k
        for a, fn in arms.items():
            t = min(res[a])
            err = ((fn().float() - ref).abs().max() / ref.abs().max()).item()
            line[a + "_us"] = round(t, 1)
            line[a + "_tflops"] = round(flop / t / 1e6, 1)
            line[a + "_relerr"] = float(f"{err:.2e}")
        line["best"] = min(arms, key=lambda a: min(res[a]))
        print(json.dumps(line), flush=True)
        del go, x, ref


if __name__ == "__main__":
    main()
