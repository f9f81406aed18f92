#!/usr/bin/env python3
"""A/B of the phase-pipelined g8p GEMM against the g256 kernel on the k-major x k-major GEMMs the
models route natively: ResNet-50 1x1 forward convolutions (NHWC pixels x Cin by Cout x Cin, bs 256)
and the transformer fused_dense forward shapes.  APEX_AMD_GEMM8P is read per call, so both arms
run in one process on the same box.  Prints one JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import apex  # noqa: E402

SHAPES = [
    # ResNet-50 1x1 fwd routed to the native GEMM (Cin = 1024): M = 256 * H * W
    (256 * 14 * 14, 256, 1024), (256 * 14 * 14, 512, 1024), (256 * 7 * 7, 2048, 1024),
    # other ResNet-50 1x1 shapes (A/B only)
    (256 * 56 * 56, 256, 64), (256 * 28 * 28, 512, 128), (256 * 7 * 7, 2048, 512),
    # transformer forward (tokens x hidden)
    (16384, 3072, 1024), (16384, 4096, 1024), (16384, 1024, 4096), (8192, 8192, 8192),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    g = apex._native.require("gemm").gemm
    os.environ["APEX_AMD_GEMM256"] = "force"
    for m, n, k in SHAPES:
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        res = {"m": m, "n": n, "k": k}
        for arm in ("1", "0"):
            os.environ["APEX_AMD_GEMM8P"] = arm
            res["g8p_ms" if arm == "1" else "g256_ms"] = round(timeit(lambda: g.linear(x, w, None, g.EPI_NONE, False)), 4)
        res["library_ms"] = round(timeit(lambda: torch.matmul(x, w.t())), 4)
        res["g8p_vs_g256"] = round(res["g256_ms"] / res["g8p_ms"], 3)
        print(json.dumps(res), flush=True)
        del x, w


if __name__ == "__main__":
    main()
