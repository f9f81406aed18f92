#!/usr/bin/env python3
"""A fixed set of the hot native kernels, 3 calls each, for rocprofv3 hardware-counter passes
(tools/gpu_pmc.sh runs one pass per counter group; tools/pmc_summary.py joins them).

Cases (bf16): fused_dense GEMM 8192^3 (256-tile LDS-DMA kernel) and GEMM+bias+GeLU 8192x3072x1024,
flash attention fwd/bwd (b16 s1024 h16 d64), LayerNorm fwd/bwd 16384x1024, NHWC BN+ReLU fwd/bwd
256x256x56x56, FusedAdam over 100M fp32 params, multi-tensor L2 norm."""
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
    g = apex._native.require("gemm").gemm
    a = torch.randn(8192, 8192, device="cuda", dtype=dt)
    w = torch.randn(8192, 8192, device="cuda", dtype=dt)
    rep(lambda: g.linear(a, w, None, g.EPI_NONE, False))
    a2 = torch.randn(8192, 1024, device="cuda", dtype=dt)
    w2 = torch.randn(3072, 1024, device="cuda", dtype=dt)
    b2 = torch.randn(3072, device="cuda", dtype=dt)
    rep(lambda: g.linear(a2, w2, b2, g.EPI_GELU, True))
    del a, w

    from apex.ops.attention import flash_attn_func

    q = torch.randn(16, 1024, 16, 64, device="cuda", dtype=dt, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True)
    v = torch.randn_like(q, requires_grad=True)
    o = flash_attn_func(q, k, v)
    go = torch.randn_like(o)
    rep(lambda: flash_attn_func(q, k, v))
    rep(lambda: torch.autograd.grad(o, (q, k, v), go, retain_graph=True))

    from apex.normalization import FusedLayerNorm

    x = torch.randn(16384, 1024, device="cuda", dtype=dt, requires_grad=True)
    ln = FusedLayerNorm(1024).cuda().to(dt)
    y = ln(x)
    gy = torch.randn_like(y)
    rep(lambda: ln(x))
    rep(lambda: torch.autograd.grad(y, [x] + list(ln.parameters()), gy, retain_graph=True))
    x4 = torch.randn(16384, 4096, device="cuda", dtype=dt, requires_grad=True)
    ln4 = FusedLayerNorm(4096).cuda().to(dt)
    y4 = ln4(x4)
    gy4 = torch.randn_like(y4)
    rep(lambda: ln4(x4))
    rep(lambda: torch.autograd.grad(y4, [x4] + list(ln4.parameters()), gy4, retain_graph=True))
    del x4, y4, gy4

    from apex.contrib.groupbn import BatchNorm2d_NHWC

    xb = torch.randn(256, 256, 56, 56, device="cuda", dtype=dt).to(memory_format=torch.channels_last)
    xb.requires_grad_(True)
    bn = BatchNorm2d_NHWC(256, fuse_relu=True, torch_channels_last=True).cuda()
    yb = bn(xb)
    gb = torch.randn_like(yb)
    rep(lambda: bn(xb))
    rep(lambda: torch.autograd.grad(yb, [xb, bn.weight, bn.bias], gb, retain_graph=True))
    del xb, yb, gb
    # the small late-stage layers (latency-bound in the step profile)
    for (nb, cb, hw) in ((256, 256, 14), (256, 2048, 7)):
        xs = torch.randn(nb, cb, hw, hw, device="cuda", dtype=dt).to(memory_format=torch.channels_last)
        xs.requires_grad_(True)
        bns = BatchNorm2d_NHWC(cb, fuse_relu=True, torch_channels_last=True).cuda()
        ys = bns(xs)
        gs = torch.randn_like(ys)
        rep(lambda: bns(xs))
        rep(lambda: torch.autograd.grad(ys, [xs, bns.weight, bns.bias], gs, retain_graph=True))

    from apex import amp_C
    from apex.optimizers import FusedAdam

    ps = [torch.randn(4096 * 1024, device="cuda", requires_grad=True) for _ in range(24)]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = FusedAdam(ps, lr=1e-3)
    rep(opt.step)
    flag = torch.zeros(1, dtype=torch.int, device="cuda")
    rep(lambda: amp_C.multi_tensor_l2norm(65536, flag, [[p.grad for p in ps]], False))
    # unscale: bf16 model grads -> fp32 master grads, and fp32 -> fp32 in place
    hs = [p.grad.to(dt) for p in ps]
    outs = [torch.empty_like(p.grad) for p in ps]
    rep(lambda: amp_C.multi_tensor_scale(65536, flag, [hs, outs], 0.5))
    rep(lambda: amp_C.multi_tensor_scale(65536, flag, [outs, outs], 0.5))
    print("pmc_kernels done", flush=True)


if __name__ == "__main__":
    main()
