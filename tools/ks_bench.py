#!/usr/bin/env python3
"""K-streamed fused 1x1 (csrc/conv/conv1x1_ks.hip) at the ResNet-50 stage-3 / 4 deep reductions:
the deferred-output forward (block output BN + shortcut + ReLU on the operand load, statistics
epilogue), the plain forward with statistics, and conv3's data gradient with bn3's dx prologue and
bn2's backward reduction.  Next to each: the unfused composition the step runs today (BN pass +
library GEMM) and a device copy of the kernel's compulsory bytes.  The column tile comes from
APEX_AMD_C1KS_NC (read once per process): run one process per setting.  One JSON line per row."""
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
    bn = apex._native.require("bn_nhwc").bn_nhwc
    dt = torch.bfloat16
    nc_env = os.environ.get("APEX_AMD_C1KS_NC", "auto")
    torch.manual_seed(0)
    for m, k, n in [(50176, 1024, 256), (12544, 2048, 512)]:
        a = torch.randn(m, k, device="cuda").to(dt)
        res = torch.randn(m, k, device="cuda").to(dt)
        w = (torch.randn(n, k, device="cuda") * 0.03).to(dt)
        wt = w.t().contiguous()
        c3 = torch.cat([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.3])
        shift = torch.randn(n, device="cuda") * 0.1
        cb = torch.cat([torch.randn(k, device="cuda"), torch.randn(k, device="cuda") * 0.1,
                        torch.randn(k, device="cuda") * 0.1])
        y2 = torch.randn(m, n, device="cuda").to(dt)
        c2 = torch.cat([torch.rand(n, device="cuda") + 0.5, torch.randn(n, device="cuda") * 0.3])
        mean2 = torch.randn(n, device="cuda") * 0.1
        big = torch.empty(3 * m * k + m * n, device="cuda", dtype=dt)
        big2 = torch.empty_like(big)
        rows = {
            "fwd_pro3_stats": (lambda: ext.bn1x1_addrelu(a, res, c3, w, shift, split=True), 3 * m * k + m * n),
            "fwd_pro0_stats": (lambda: ext.bn1x1(a, w, False, None, shift, True), m * k + m * n),
            "dgrad_pro2_red": (lambda: ext.dgrad_bnred(a, wt, None, None, y2, mean2, coef=c2, py=res, pcoef=cb,
                                                       want_aout=True), 3 * m * k + 2 * m * n),
            "ref_apply+mm": (lambda: torch.matmul(bn.apply(a, res, c3, True, True)[0].view(m, k), w.t()), None),
            "ref_bwd_apply+mm": (lambda: torch.matmul(bn.bwd_apply(a, res, c3, cb), wt), None),
            "ref_mm": (lambda: torch.matmul(a, w.t()), None),
        }
        for name, (fn, elems) in rows.items():
            us = timeit(fn)
            row = {"m": m, "k": k, "n": n, "nc": nc_env, "op": name, "us": round(us, 1)}
            if elems:
                row["tb_s"] = round(elems * 2 / us / 1e6, 2)
                cp = timeit(lambda: big2[: elems // 2].copy_(big[: elems // 2]))  # same bytes moved (r + w)
                row["copy_us"] = round(cp, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
