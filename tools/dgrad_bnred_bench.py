#!/usr/bin/env python3
"""conv1's data gradient in the linked ResNet-50 node (csrc/conv/conv1x1_bn.hip dgrad form: the
block below's output ReLU bits mask the sum of the 1x1 data gradient and the shortcut gradient,
and that block's bn3 backward sums accumulate in the epilogue) at every stage's shape, alone in a
process, next to a device copy of the kernel's compulsory bytes.  One JSON line per shape."""
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


def main():
    import apex

    ext = apex._native.require("conv").conv
    dt = torch.bfloat16
    torch.manual_seed(0)
    # (pixels, conv1 output channels = reduction depth, block channels = output columns)
    for m, k, n in [(802816, 64, 256), (200704, 128, 512), (50176, 256, 1024), (12544, 512, 2048),
                    (50176, 512, 1024)]:
        g = torch.randn(m, k, device="cuda").to(dt)
        w = (torch.randn(k, n, device="cuda") * 0.03).to(dt)
        short = torch.randn(m, n, device="cuda").to(dt)
        x = torch.randn(m, n, device="cuda").to(dt)
        bits = torch.randint(0, 256, (m * n // 8,), device="cuda", dtype=torch.uint8)
        mean = torch.randn(n, device="cuda") * 0.1
        us = timeit(lambda: ext.dgrad_bnred(g, w, short, bits, x, mean))
        elems = m * k + 3 * m * n  # g, short, x read; dx written (bits: 1/16 more)
        big = torch.empty(elems // 2 + 8, device="cuda", dtype=dt)
        big2 = torch.empty_like(big)
        cp = timeit(lambda: big2.copy_(big))
        mm = timeit(lambda: torch.matmul(g, w))
        print(json.dumps({"m": m, "k": k, "n": n, "us": round(us, 1), "tb_s": round(elems * 2 / us / 1e6, 2),
                          "copy_same_bytes_us": round(cp, 1), "torch_mm_us": round(mm, 1)}), flush=True)


if __name__ == "__main__":
    main()
