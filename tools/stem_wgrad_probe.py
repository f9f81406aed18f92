#!/usr/bin/env python3
"""Time the native stem weight-gradient kernel alone at bs 256 (diagnostic modes through
APEX_AMD_STEM_WG_MODE, csrc/conv/stem.hip) and the conv3 backward kernel; one JSON line each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timeit(fn, iters=10, warmup=3):
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
    torch.manual_seed(0)
    dt = torch.bfloat16
    x = torch.randn(256, 3, 224, 224, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).to(dt).contiguous(memory_format=torch.channels_last)
    rm = torch.zeros(64, device="cuda")
    y, part, xp = ext.stem_fprop(x, w, rm)
    m = float(y.size(0) * y.size(2) * y.size(3))
    g = torch.ones(64, device="cuda")
    b = torch.zeros(64, device="cuda")
    sm, si, coef = ext.bn_finalize(part, m, rm, g, b, rm.clone(), torch.ones(64, device="cuda"), 1e-5, 0.1)
    p, idx = ext.stem_pool(y, coef)
    dp = torch.randn_like(p)
    part2 = ext.stem_reduce(dp, idx, y, coef, sm)
    cb, gg, gb = ext.bnbwd_finalize(part2, m, sm, si, g)
    us = timeit(lambda: ext.stem_wgrad(dp, idx, y, coef, cb.view(-1), xp, w))
    print(json.dumps({"kernel": "stem_wgrad", "mode": int(os.environ.get("APEX_AMD_STEM_WG_MODE", "0")),
                      "us": round(us, 1)}))


if __name__ == "__main__":
    main()
