#!/usr/bin/env python3
"""GEMM routes at the GPT-2 medium / BERT-large dense-layer shapes (16384 tokens, hidden 1024):
torch.matmul (hipBLASLt, heuristic's first answer) vs the hipBLASLt wrapper with per-shape top-8
timing (lt_gemm.mm) vs the native MFMA GEMM (gemm.matmul), for the forward (x W^T), data-gradient
(g W) and weight-gradient (g^T x) products.  One JSON line per (shape, op).
Run on the GPU box: python tools/gemm_route_bench.py [--tokens 16384]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


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


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    args = ap.parse_args()
    import apex  # noqa: F401
    from apex import _native

    lt = _native.require("lt_gemm").lt_gemm
    g = _native.require("gemm").gemm
    dt = torch.bfloat16
    M = args.tokens
    torch.manual_seed(0)
    for (n, k) in [(3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)]:
        x = torch.randn(M, k, device="cuda", dtype=dt)
        w = torch.randn(n, k, device="cuda", dtype=dt) * 0.03
        gy = torch.randn(M, n, device="cuda", dtype=dt)
        ops = {
            "fwd": (lambda: x.matmul(w.t()), lambda: lt.mm(x, w, False, True),
                    lambda: g.matmul(x, True, w, True, M, n, k, 0, None, None, False)[0]),
            "dgrad": (lambda: gy.matmul(w), lambda: lt.mm(gy, w, False, False),
                      lambda: g.matmul(gy, True, w, False, M, k, n, 0, None, None, False)[0]),
            "wgrad": (lambda: gy.t().matmul(x), lambda: lt.mm(gy, x, True, False),
                      lambda: g.matmul(gy, False, x, False, n, k, M, 0, None, None, False)[0]),
        }
        for op, (ft, fl, fn) in ops.items():
            ref = ft()
            flop = 2.0 * M * n * k
            row = {"tokens": M, "n": n, "k": k, "op": op}
            for name, f in (("torch", ft), ("lt_top8", fl), ("native", fn)):
                try:
                    out = f()
                    if isinstance(out, list):
                        if not out:
                            row[name] = "unsupported"
                            continue
                        out = out[0]
                        f0 = f
                        f = (lambda f0=f0: f0()[0])
                    us = timeit(f)
                    row[name + "_us"] = round(us, 1)
                    row[name + "_tflops"] = round(flop / us / 1e6, 1)
                    row[name + "_rel"] = round(rel(out, ref), 5)
                except Exception as exc:  # noqa: BLE001
                    row[name] = "error: " + str(exc)[:120]
            print(json.dumps(row), flush=True)
    print(json.dumps({"plans": [list(p) for p in lt.plan_table()]}))


if __name__ == "__main__":
    main()
