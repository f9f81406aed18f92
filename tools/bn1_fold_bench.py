#!/usr/bin/env python3
"""Per-kernel cost of the bn1 fold (ops/bottleneck_bn.py _bn1_fold): the stride-1 3x3 forward and
weight gradient with and without the BN + ReLU input prologue, and the apply pass it replaces, at
the ResNet-50 shapes it takes (bs 256, bf16).  One JSON line per row."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


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
    import apex
    from apex.ops import conv as C

    bn = apex._native.require("bn_nhwc").bn_nhwc
    dt = torch.bfloat16
    for (c, h) in [(64, 56), (512, 7)]:
        n = 256
        y = torch.randn(n, c, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).to(dt).contiguous(memory_format=torch.channels_last)
        gy = torch.randn(n, c, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        coef = torch.cat([torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.5])
        shift = torch.zeros(c, device="cuda")
        y2 = y.permute(0, 2, 3, 1).reshape(-1, c)
        z = bn.apply(y2, None, coef, True)[0].view(n, h, h, c).permute(0, 3, 1, 2)
        rows = {
            "apply": timeit(lambda: bn.apply(y2, None, coef, True)),
            "fwd_plain": timeit(lambda: C.conv_tap_forward(z, w, 1, 1, stats_shift=shift)),
            "fwd_pro": timeit(lambda: C.conv_tap_forward(y, w, 1, 1, stats_shift=shift, pcoef=coef)),
            "wgrad_plain": timeit(lambda: C.conv_tap_wgrad(gy, z, w.shape, 1, 1, dt)),
            "wgrad_pro": timeit(lambda: C.conv_tap_wgrad(gy, y, w.shape, 1, 1, dt, xcoef=coef)),
        }
        print(json.dumps({"shape": f"{h}x{h}x{c}", **{k: round(v, 1) for k, v in rows.items()}}), flush=True)


if __name__ == "__main__":
    main()
