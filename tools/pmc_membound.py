#!/usr/bin/env python3
"""Memory-bound kernels for a rocprofv3 counter pass WITH their own roof in the same run: a plain
elementwise copy (torch.mul by 1, the fp32 Adam step's byte count) is profiled beside FusedAdam (fp32, 24 x 4M params),
the multi-tensor L2 norm and scale, and LayerNorm forward / backward at hidden 1024, 4096, 32768 and
65536 (16M elements each), so
every kernel's FETCH+WRITE rate can be read against the copy rate under the same profiler clock
(profiled passes run at ~1.9 GHz vs ~2.0 un-profiled).  3 calls each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import apex  # noqa: E402


def rep(fn, n=3):
    for _ in range(n):
        fn()
    torch.cuda.synchronize()


def main():
    dt = torch.bfloat16
    # the roof: an elementwise kernel moving the same bytes as the fp32 Adam step below (24 x 4M
    # params x 28 B = 2.68 GB: 1.34 GB read + 1.34 GB written; a same-dtype copy_ would go to the
    # DMA engine, not a kernel)
    src = torch.empty(24 * 4096 * 1024 * 28 // 8, device="cuda", dtype=torch.float32).uniform_()
    dst = torch.empty_like(src)
    rep(lambda: torch.mul(src, 1.0, out=dst))
    del src, dst

    from apex import amp_C
    from apex.optimizers import FusedAdam

    ps = [torch.randn(4096 * 1024, device="cuda", requires_grad=True) for _ in range(24)]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = FusedAdam(ps, lr=1e-3)
    rep(opt.step)
    flag = torch.zeros(1, dtype=torch.int, device="cuda")
    rep(lambda: amp_C.multi_tensor_l2norm(65536, flag, [[p.grad for p in ps]], False))
    hs = [p.grad.to(dt) for p in ps]
    outs = [torch.empty_like(p.grad) for p in ps]
    rep(lambda: amp_C.multi_tensor_scale(65536, flag, [hs, outs], 0.5))
    rep(lambda: amp_C.multi_tensor_scale(65536, flag, [outs, outs], 0.5))
    del ps, hs, outs, opt

    from apex.normalization import FusedLayerNorm

    for hid in (1024, 4096, 32768, 65536):
        x = torch.randn(16384 * 1024 // hid, hid, device="cuda", dtype=dt, requires_grad=True)
        ln = FusedLayerNorm(hid).cuda().to(dt)
        y = ln(x)
        gy = torch.randn_like(y)
        rep(lambda: ln(x))
        rep(lambda: torch.autograd.grad(y, [x] + list(ln.parameters()), gy, retain_graph=True))
    print("pmc_membound done", flush=True)


if __name__ == "__main__":
    main()
