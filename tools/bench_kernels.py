#!/usr/bin/env python3
"""Kernel-level benchmarks on one MI355X: gfx950 native kernels vs the stock PyTorch-ROCm path
(hipBLASLt GEMM, MIOpen BN, torch LayerNorm / softmax / Adam).  Prints one JSON line per case:
time per call (median of N), achieved TFLOP/s or GB/s, and the ratio to the stock op.

Usage (GPU box): python tools/bench_kernels.py [--only gemm,ln,softmax,bn,adam] > gpurun_out/kernels.jsonl
"""
import argparse
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
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_gemm():
    import apex

    g = apex._native.require("gemm").gemm
    dt = torch.bfloat16
    shapes = [(8192, 8192, 8192), (4096, 4096, 4096), (16384, 4096, 1024), (16384, 1024, 4096),
              (8192, 3072, 1024), (8192, 1024, 3072)]
    for (m, n, k) in shapes:
        a = torch.randn(m, k, device="cuda", dtype=dt)
        w = torch.randn(n, k, device="cuda", dtype=dt)
        flops = 2.0 * m * n * k
        t_ours = timeit(lambda: g.linear(a, w, None, g.EPI_NONE, False))
        os.environ["APEX_AMD_GEMM256"] = "off"
        t_128 = timeit(lambda: g.linear(a, w, None, g.EPI_NONE, False))
        os.environ.pop("APEX_AMD_GEMM256")
        t_ref = timeit(lambda: torch.matmul(a, w.t()))
        emit(kernel="gemm_fwd_nt", m=m, n=n, k=k, ms=t_ours, tflops=flops / t_ours / 1e9, tile128_tflops=flops / t_128 / 1e9,
             hipblaslt_ms=t_ref, hipblaslt_tflops=flops / t_ref / 1e9, speedup=t_ref / t_ours)
        dy = torch.randn(m, n, device="cuda", dtype=dt)
        t_ours = timeit(lambda: g.linear_dgrad(dy, w, g.EPI_NONE, None))
        t_ref = timeit(lambda: torch.matmul(dy, w))
        emit(kernel="gemm_dgrad_nn", m=m, n=k, k=n, ms=t_ours, tflops=flops / t_ours / 1e9, hipblaslt_ms=t_ref,
             speedup=t_ref / t_ours)
        t_ours = timeit(lambda: g.linear_wgrad(dy, a))
        t_nosplit = _with_env("APEX_AMD_SPLITK", "off", lambda: timeit(lambda: g.linear_wgrad(dy, a)))
        t_ref = timeit(lambda: torch.matmul(dy.t(), a))
        emit(kernel="gemm_wgrad_tn", m=n, n=k, k=m, ms=t_ours, tflops=flops / t_ours / 1e9, hipblaslt_ms=t_ref,
             speedup=t_ref / t_ours, no_splitk_ms=t_nosplit)
        b = torch.randn(n, device="cuda", dtype=dt)
        t_ours = timeit(lambda: g.linear(a, w, b, g.EPI_GELU, True))
        t_ref = timeit(lambda: torch.nn.functional.gelu(torch.addmm(b, a, w.t()), approximate="tanh"))
        emit(kernel="gemm_bias_gelu_aux", m=m, n=n, k=k, ms=t_ours, tflops=flops / t_ours / 1e9, torch_ms=t_ref,
             speedup=t_ref / t_ours)


def bench_dense_route():
    """FusedDense / FusedDenseGeluDense forward+backward per shape: native kernels, library
    GEMMs (hipBLASLt) and the measured per-shape routing."""
    from apex.fused_dense import FusedDense, FusedDenseGeluDense
    from apex.fused_dense import fused_dense as fd

    dt = torch.bfloat16
    for (tokens, hin, hout) in [(16384, 1024, 3072), (16384, 1024, 4096), (16384, 4096, 1024), (8192, 1024, 1024)]:
        x = torch.randn(tokens, hin, device="cuda", dtype=dt, requires_grad=True)
        m = FusedDense(hin, hout).cuda().to(dt)
        gy = torch.randn(tokens, hout, device="cuda", dtype=dt)
        res = {}
        for mode in ("native", "library", "auto"):
            os.environ["APEX_AMD_DENSE_ROUTE"] = mode
            res[mode] = timeit(lambda: torch.autograd.backward(m(x), gy))
        os.environ.pop("APEX_AMD_DENSE_ROUTE")
        emit(kernel="fused_dense_fwd_bwd", tokens=tokens, k=hin, n=hout, native_ms=res["native"],
             library_ms=res["library"], routed_ms=res["auto"], routed_vs_library=res["library"] / res["auto"],
             routes={"/".join(map(str, k)): v for k, v in fd.route_table().items()
                     if k[1:4] == (tokens, hout, hin)})
    for (tokens, h, f) in [(16384, 1024, 4096)]:
        x = torch.randn(tokens, h, device="cuda", dtype=dt, requires_grad=True)
        m = FusedDenseGeluDense(h, f, h).cuda().to(dt)
        gy = torch.randn(tokens, h, device="cuda", dtype=dt)
        res = {}
        for mode in ("native", "library", "auto"):
            os.environ["APEX_AMD_DENSE_ROUTE"] = mode
            res[mode] = timeit(lambda: torch.autograd.backward(m(x), gy))
        os.environ.pop("APEX_AMD_DENSE_ROUTE")
        emit(kernel="fused_dense_gelu_dense_fwd_bwd", tokens=tokens, h=h, ffn=f, native_ms=res["native"],
             library_ms=res["library"], routed_ms=res["auto"], routed_vs_library=res["library"] / res["auto"])


def bench_ln():
    from apex.normalization import FusedLayerNorm

    for (n1, n2) in [(16384, 1024), (8192, 4096), (4096, 8192), (32768, 768)]:
        x = torch.randn(n1, n2, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        m = FusedLayerNorm(n2).cuda().to(torch.bfloat16)
        ref = torch.nn.LayerNorm(n2).cuda().to(torch.bfloat16)
        gy = torch.randn_like(x)
        nbytes = x.numel() * 2 * 2
        t = timeit(lambda: m(x))
        tr = timeit(lambda: ref(x))
        emit(kernel="layer_norm_fwd", n1=n1, n2=n2, ms=t, gbps=nbytes / t / 1e6, torch_ms=tr, speedup=tr / t)
        y = m(x)
        yr = ref(x)
        t = timeit(lambda: torch.autograd.grad(y, [x] + list(m.parameters()), gy, retain_graph=True))
        tr = timeit(lambda: torch.autograd.grad(yr, [x] + list(ref.parameters()), gy, retain_graph=True))
        emit(kernel="layer_norm_bwd", n1=n1, n2=n2, ms=t, gbps=x.numel() * 2 * 3 / t / 1e6, torch_ms=tr,
             speedup=tr / t)


def bench_softmax():
    from apex.transformer.functional.fused_softmax import scaled_masked_softmax, scaled_upper_triang_masked_softmax

    for (b, h, s) in [(8, 16, 1024), (4, 16, 2048), (2, 16, 4096)]:
        x = torch.randn(b, h, s, s, device="cuda", dtype=torch.bfloat16)
        mask = torch.rand(b, 1, s, s, device="cuda") < 0.1
        t = timeit(lambda: scaled_masked_softmax(x, mask, 0.125))
        tr = timeit(lambda: torch.softmax((x * 0.125).masked_fill(mask, -10000.0).float(), -1).to(x.dtype))
        emit(kernel="scaled_masked_softmax_fwd", b=b, h=h, s=s, ms=t, gbps=x.numel() * 4 / t / 1e6, torch_ms=tr,
             speedup=tr / t)
        xc = x.view(-1, s, s)
        t = timeit(lambda: scaled_upper_triang_masked_softmax(x, None, 0.125))
        emit(kernel="causal_softmax_fwd", b=b, h=h, s=s, ms=t, gbps=x.numel() * 3 / t / 1e6)
        del xc


def bench_bn():
    from apex.contrib.groupbn import BatchNorm2d_NHWC

    for (n, c, hw) in [(256, 64, 112), (256, 256, 56), (256, 512, 28), (256, 1024, 14), (256, 2048, 7)]:
        x = torch.randn(n, c, hw, hw, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        ours = BatchNorm2d_NHWC(c, fuse_relu=True, torch_channels_last=True).cuda()
        ref = torch.nn.BatchNorm2d(c).cuda()
        gy = torch.randn_like(x)
        t = timeit(lambda: ours(x))
        tr = timeit(lambda: torch.relu(ref(x)))
        emit(kernel="bn_relu_fwd_nhwc", n=n, c=c, hw=hw, ms=t, gbps=x.numel() * 2 * 3 / t / 1e6, torch_ms=tr,
             speedup=tr / t)
        y = ours(x)
        yr = torch.relu(ref(x))
        t = timeit(lambda: torch.autograd.grad(y, [x, ours.weight, ours.bias], gy, retain_graph=True))
        tr = timeit(lambda: torch.autograd.grad(yr, [x, ref.weight, ref.bias], gy, retain_graph=True))
        emit(kernel="bn_relu_bwd_nhwc", n=n, c=c, hw=hw, ms=t, gbps=x.numel() * 2 * 5 / t / 1e6, torch_ms=tr,
             speedup=tr / t)


def bench_adam():
    from apex.optimizers import FusedAdam

    sizes = [4096 * 1024] * 24 + [1024] * 48  # ~100M params
    ps = [torch.randn(s, device="cuda", requires_grad=True) for s in sizes]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = FusedAdam(ps, lr=1e-3)
    ps2 = [p.detach().clone().requires_grad_(True) for p in ps]
    for p, q in zip(ps, ps2):
        q.grad = p.grad.clone()
    ref = torch.optim.AdamW(ps2, lr=1e-3, fused=True)
    n = sum(sizes)
    t = timeit(opt.step)
    tr = timeit(ref.step)
    nbytes = n * 4 * 7  # read g, p, m, v; write p, m, v
    emit(kernel="fused_adam_fp32", params=n, ms=t, gbps=nbytes / t / 1e6, torch_fused_ms=tr, speedup=tr / t)


def _with_env(name, value, fn):
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        return fn()
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old


def bench_attn():
    """flash fwd / bwd vs torch SDPA; the kernel variants are timed side by side
    (fwd: lazy O-rescale on/off; bwd: split atomic-free kernels vs the fused dQ-atomic kernel)."""
    from apex.ops.attention import flash_attn_func
    import torch.nn.functional as F

    for (b, s, h, d, causal) in [(16, 1024, 16, 64, False), (8, 2048, 16, 128, False), (8, 2048, 16, 128, True),
                                 (4, 4096, 32, 128, True), (32, 512, 16, 64, False)]:
        q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn_like(q, requires_grad=True)
        v = torch.randn_like(q, requires_grad=True)
        flops = 4.0 * b * h * s * s * d * (0.5 if causal else 1.0)
        fwd = lambda: flash_attn_func(q, k, v, causal=causal)  # noqa: E731
        t = timeit(fwd)
        var = {"qf2_ms": _with_env("APEX_ATTN_FWD_QF", "2", lambda: timeit(fwd)),
               "occ_lo_ms": _with_env("APEX_ATTN_FWD_OCC", "lo", lambda: timeit(fwd))}
        qt, kt, vt = (x.detach().transpose(1, 2).contiguous().requires_grad_(True) for x in (q, k, v))
        tr = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
        emit(kernel="flash_fwd", b=b, s=s, h=h, d=d, causal=causal, ms=t, tflops=flops / t / 1e9, sdpa_ms=tr,
             sdpa_tflops=flops / tr / 1e9, speedup=tr / t, **var)
        o = flash_attn_func(q, k, v, causal=causal)
        g = torch.randn_like(o)
        bwd = lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True)  # noqa: E731
        t = timeit(bwd)
        var = {f"{m}_ms": _with_env("APEX_ATTN_BWD", m, lambda: timeit(bwd)) for m in ("split", "atomic")}
        orr = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
        gt = g.transpose(1, 2).contiguous()
        tr = timeit(lambda: torch.autograd.grad(orr, (qt, kt, vt), gt, retain_graph=True))
        emit(kernel="flash_bwd", b=b, s=s, h=h, d=d, causal=causal, ms=t, tflops=2.5 * flops / t / 1e9, sdpa_ms=tr,
             sdpa_tflops=2.5 * flops / tr / 1e9, speedup=tr / t, **var)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="attn,gemm,ln,softmax,bn,adam,dense_route")
    a = ap.parse_args()
    torch.manual_seed(0)
    for name in a.only.split(","):
        globals()["bench_" + name]()


if __name__ == "__main__":
    main()
