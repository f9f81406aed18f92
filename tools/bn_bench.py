#!/usr/bin/env python3
"""Fused NHWC BN passes at the ResNet-50 (bs 256) shapes: time and effective HBM GB/s of the
forward (stats + apply) and backward (reduce + apply) of ``_C.bn_nhwc``, one JSON line per case.
Tuning knobs (APEX_BN_STATS_BPC, APEX_BN_BWD_BPC: workgroups per CU of the partial passes) are read from the environment.
Run on the GPU box: python tools/bn_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    return s.elapsed_time(e) / iters


def main():
    import apex

    ext = apex._native._C.bn_nhwc
    # (hw, C, kind): kind "relu" = conv->BN->ReLU, "zrelu2" = block output BN + residual + ReLU whose
    # output forks into two consumers (two incoming gradients, grad_z needed)
    cases = [(112, 64, "relu"), (56, 64, "relu"), (56, 256, "zrelu2"), (56, 256, "plain"), (28, 128, "relu"),
             (28, 512, "zrelu2"), (14, 256, "relu"), (14, 1024, "zrelu2"), (7, 512, "relu"), (7, 2048, "zrelu2")]
    knobs = {k: os.environ.get(k) for k in ("APEX_BN_STATS_BPC", "APEX_BN_BWD_BPC")}
    tot_f = tot_b = 0.0
    for hw, c, kind in cases:
        m = 256 * hw * hw
        dev = "cuda"
        x = torch.randn(m, c, device=dev, dtype=torch.bfloat16)
        z = torch.randn(m, c, device=dev, dtype=torch.bfloat16) if kind == "zrelu2" else None
        w = torch.rand(c, device=dev) + 0.5
        b = torch.randn(c, device=dev) * 0.1
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        relu = kind != "plain"
        bits = z is not None and os.environ.get("APEX_BN_BITS", "1") != "0"
        y, sm, si, coef, mask = ext.fwd_train(x, z, w, b, rm, rv, 0.1, 1e-5, relu, bits)
        tf = timeit(lambda: ext.fwd_train(x, z, w, b, rm, rv, 0.1, 1e-5, relu, bits))
        dy = torch.randn_like(x)
        dy2 = torch.randn_like(x) if kind == "zrelu2" else None
        need_dz = kind == "zrelu2"
        zb = None if bits else z
        tb = timeit(lambda: ext.bwd(dy, x, zb, w, sm, si, coef, relu, need_dz, dy2, mask if bits else None))
        e = m * c * 2
        nf = 3 + (1 if z is not None else 0)
        # bwd passes: reduce reads dy[,dy2],x[,z] (+writes dz); apply reads dy|dz, x [,z], writes dx
        if kind == "zrelu2":
            nb = 5 + 3
        elif kind == "relu":
            nb = 2 + 3
        else:
            nb = 2 + 3
        tot_f += tf
        tot_b += tb
        print(json.dumps(dict(hw=hw, c=c, kind=kind, fwd_ms=round(tf, 4), bwd_ms=round(tb, 4),
                              fwd_gbps=round(e * nf / tf / 1e6), bwd_gbps=round(e * nb / tb / 1e6), **knobs)),
              flush=True)
    print(json.dumps(dict(total_fwd_ms=round(tot_f, 3), total_bwd_ms=round(tot_b, 3), **knobs)), flush=True)


if __name__ == "__main__":
    main()
