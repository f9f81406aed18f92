"""Stride-2 3x3 weight gradient at ResNet-50's downsampling shapes (bs 256, bf16, channels_last):
the halo-tile kernel's stride-2 form (csrc/conv/conv3x3_wgrad.hip) vs MIOpen's
(aten.convolution_backward, weight only).  One JSON line per (shape, engine).

    python tools/wgrad_s2_bench.py [--batch 256] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(56, 128, 128), (28, 256, 256), (14, 512, 512)]  # input h = w, cin, cout


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from apex.ops import conv as C

    dt = torch.bfloat16
    for h, cin, cout in SHAPES:
        torch.manual_seed(0)
        x = torch.randn(args.batch, cin, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        gy = torch.randn(args.batch, cout, h // 2, h // 2, device="cuda").to(dt).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 3, 3, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        nat = lambda: C.conv_tap_wgrad(gy, x, w.shape, 2, 1, dt)  # noqa: E731
        lib = lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [2, 2], [1, 1], [1, 1], False,  # noqa: E731
                                                          [0, 0], 1, [False, True, False])[1]
        ref = lib().float()
        got = nat().float()
        rel = float((got - ref).abs().max() / ref.abs().max())
        flop = 2.0 * args.batch * (h // 2) ** 2 * cout * cin * 9
        for name, fn in (("native_halo_s2", nat), ("miopen", lib)):
            us = _time(fn, args.iters)
            print(json.dumps({"in_hw": h, "cin": cin, "cout": cout, "batch": args.batch, "engine": name,
                              "us": round(us, 1), "tflops": round(flop / us / 1e6, 1), "rel_vs_miopen": rel}),
                  flush=True)


if __name__ == "__main__":
    main()
