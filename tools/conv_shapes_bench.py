#!/usr/bin/env python3
"""Per-shape cost of every ResNet-50 convolution (bs 256, bf16, channels_last) through
MIOpen (torch.nn.functional.conv2d / convolution_backward): forward, dgrad and wgrad timed
separately, each against its roofline = max(bytes / 6.3 TB/s, FLOPs / 2.5 PF).  One JSON line per
shape plus a totals line weighted by how many times the shape occurs in the network.
Run on the GPU box: python tools/conv_shapes_bench.py [--batch 256]"""
import argparse
import json

import torch
import torch.nn.functional as F

HBM = 6.3e12
MFMA = 2.5e15

# (cin, cout, k, stride, h_in, count in ResNet-50)
SHAPES = [
    (3, 64, 7, 2, 224, 1),
    (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3),
    (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1), (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1),
    (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
    (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
]


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
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    B = a.batch
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "roof_fwd": 0.0, "roof_dgrad": 0.0, "roof_wgrad": 0.0}
    for cin, cout, k, st, h, cnt in SHAPES:
        pad = k // 2
        ho = (h + 2 * pad - k) // st + 1
        x = torch.randn(B, cin, h, h, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last)
        gy = torch.randn(B, cout, ho, ho, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        args = ([st, st], [pad, pad], [1, 1], False, [0, 0], 1)
        t_f = timeit(lambda: F.conv2d(x, w, None, st, pad))
        t_d = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, *args, [True, False, False]))
        t_w = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, *args, [False, True, False]))
        flops = 2.0 * B * ho * ho * cout * cin * k * k
        bx, by, bw = x.numel() * 2, gy.numel() * 2, w.numel() * 2
        roof = lambda byts: max(byts / HBM, flops / MFMA)  # noqa: E731
        r = {"cin": cin, "cout": cout, "k": k, "stride": st, "h": h, "count": cnt,
             "fwd_us": round(t_f * 1e6, 1), "dgrad_us": round(t_d * 1e6, 1), "wgrad_us": round(t_w * 1e6, 1),
             "roof_fwd_us": round(roof(bx + by + bw) * 1e6, 1), "roof_dgrad_us": round(roof(bx + by + bw) * 1e6, 1),
             "roof_wgrad_us": round(roof(bx + by + bw) * 1e6, 1), "gflop": round(flops / 1e9, 1),
             "mbytes_io": round((bx + by) / 1e6, 1)}
        for key in ("fwd", "dgrad", "wgrad"):
            tot[key] += cnt * r[key + "_us"] / 1e3
            tot["roof_" + key] += cnt * r["roof_" + key + "_us"] / 1e3
        print(json.dumps(r), flush=True)
        del x, w, gy
    print(json.dumps({"total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
