#!/usr/bin/env python3
"""ResNet-50 stage-1 3x3 convolution (bs 256, 56 x 56, 64 -> 64, bf16): the spatial-tile kernel
(conv3x3_sp.hip, tile configuration 21) against the tap-GEMM fprop2 configuration it replaces
(cfg 7) and MIOpen, forward with the BN statistics epilogue and the data gradient.  One JSON line
per arm.  Run on the GPU box: python tools/conv_sp_bench.py [--batch 256]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, iters=20, warmup=5):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hw", type=int, default=56)
    args = ap.parse_args()
    import apex  # noqa: F401
    from apex.ops import conv as C

    torch.backends.cudnn.benchmark = True
    n, h = args.batch, args.hw
    x = torch.randn(n, 64, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, 64, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    shift = torch.zeros(64, device="cuda")
    flop = 2.0 * n * h * h * 64 * 64 * 9
    ext = C._conv_ext()
    for name, cfg in (("spatial", 21), ("fprop2_cfg7", 7)):
        ext.force_fprop_cfg(cfg)
        try:
            f = timeit(lambda: C.conv_tap_forward(x, w, 1, 1, stats_shift=shift))
            d = timeit(lambda: C.conv_tap_dgrad(gy, w, x.shape, 1, 1))
        finally:
            ext.force_fprop_cfg(-1)
        print(json.dumps({"arm": name, "fwd_stats_us": round(f, 1), "dgrad_us": round(d, 1),
                          "fwd_tflops": round(flop / f / 1e6, 1), "dgrad_tflops": round(flop / d / 1e6, 1),
                          "batch": n, "hw": h}), flush=True)
    f = timeit(lambda: F.conv2d(x, w, None, 1, 1))
    print(json.dumps({"arm": "miopen", "fwd_us": round(f, 1), "fwd_tflops": round(flop / f / 1e6, 1), "batch": n,
                      "hw": h}), flush=True)


if __name__ == "__main__":
    main()
