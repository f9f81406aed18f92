#!/usr/bin/env python3
"""ResNet-50 stage-1 conv3 backward (M = 802,816 pixels, C4 = 256, W = 64, bf16): the fused kernel
(csrc/conv/conv3_bwd.hip) against the two-kernel path it replaces (dgrad with the bn3-dx prologue
and bn2 reduction writing dx3, then the weight gradient re-reading dx3).  One JSON line per row."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
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
    import apex  # noqa: F401
    from apex import _native

    ext = _native.require("conv").conv
    dt, dev = torch.bfloat16, "cuda"
    m, c4, w = 256 * 56 * 56, 256, 64
    torch.manual_seed(0)
    dm = torch.randn(m, c4, device=dev).to(dt)
    y3 = torch.randn(m, c4, device=dev).to(dt)
    y2 = torch.randn(m, w, device=dev).to(dt)
    w3 = (torch.randn(c4, w, device=dev) * 0.1).to(dt)
    cb3 = torch.randn(3 * c4, device=dev) * 0.5
    c2 = torch.cat([torch.rand(w, device=dev) + 0.5, torch.randn(w, device=dev) * 0.3])
    mean2 = torch.randn(w, device=dev) * 0.1

    def fused():
        return ext.conv3_bwd(dm, y3, y2, w3, cb3, c2, mean2)

    def unfused():
        dz2, part2, dx3 = ext.dgrad_bnred(dm, w3, None, None, y2, mean2, coef=c2, py=y3, pcoef=cb3, want_aout=True)
        return ext.wgrad1x1(dx3, y2, c2, dt)

    hbm = (2 * m * c4 + 2 * m * w) * 2
    for name, fn in (("fused", fused), ("unfused_dgrad+wgrad", unfused)):
        us = timeit(fn)
        print(json.dumps({"row": name, "us": round(us, 1), "m": m, "c4": c4, "w": w,
                          "fused_min_bytes_TBps": round(hbm / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
