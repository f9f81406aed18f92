"""Forward + backward time of the frozen-BN Bottleneck: native conv + scale/bias/residual/ReLU
epilogue kernels (``use_native=True``) vs the BN folded into MIOpen convs (``use_native=False``).

ResNet-50 stage shapes at batch 64, channels_last bf16.  One JSON line per (shape, variant).
Usage: python tools/bottleneck_bench.py [--batch 64] [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from apex.contrib.bottleneck import Bottleneck  # noqa: E402

SHAPES = [  # (cin, bottleneck, cout, stride, H)
    (256, 64, 256, 1, 56),
    (256, 128, 512, 2, 56),
    (512, 128, 512, 1, 28),
    (512, 256, 1024, 2, 28),
    (1024, 256, 1024, 1, 14),
    (2048, 512, 2048, 1, 7),
]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    for cin, mid, cout, stride, h in SHAPES:
        torch.manual_seed(0)
        blk = Bottleneck(cin, mid, cout, stride=stride, use_cudnn=True).cuda().to(torch.bfloat16)
        blk = blk.to(memory_format=torch.channels_last)
        x = torch.randn(args.batch, cin, h, h, device="cuda", dtype=torch.bfloat16)
        x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
        for native in (True, False):
            blk.use_native = native

            def fwd():
                with torch.no_grad():
                    blk(x)

            def fwd_bwd():
                y = blk(x)
                y.backward(torch.ones_like(y))

            row = {"shape": [cin, mid, cout, stride, h], "batch": args.batch,
                   "variant": "native_epilogue" if native else "folded_miopen",
                   "fwd_ms": round(timed(fwd, args.iters), 4), "fwd_bwd_ms": round(timed(fwd_bwd, args.iters), 4)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
