#!/usr/bin/env python3
"""LayerNorm forward / backward bandwidth at wide hidden sizes (fast path up to 65536, 16-wave
rows) against torch.nn.functional.layer_norm; bf16 in/out, bf16 gamma/beta.  Bytes counted are
the minimum the op must move: fwd x + y, bwd x + dy + dx (gamma / beta / statistics excluded).
One JSON line per (hidden, pass).  Run on the GPU box: python tools/ln_wide_bench.py"""
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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    from apex.normalization import FusedLayerNorm

    dt = torch.bfloat16
    rows_bytes = 256 << 20  # 256 MiB of activations per tensor
    copy_src = torch.empty(rows_bytes // 2, device="cuda", dtype=dt)
    copy_dst = torch.empty_like(copy_src)
    t_copy = timeit(lambda: copy_dst.copy_(copy_src))
    print(json.dumps({"row": "copy", "bytes": 2 * rows_bytes, "us": round(t_copy, 1),
                      "GBps": round(2 * rows_bytes / t_copy / 1e3, 1)}), flush=True)
    for hidden in (1024, 4096, 8192, 12288, 16384, 32768, 65536):
        n1 = rows_bytes // (2 * hidden)
        x = torch.randn(n1, hidden, device="cuda", dtype=dt)
        m = FusedLayerNorm(hidden).cuda().to(dt)
        w, b = m.weight, m.bias
        g = torch.randn_like(x)
        xr = x.detach().requires_grad_(True)
        for impl in ("apex", "torch"):
            if impl == "apex":
                f = lambda: m(x)  # noqa: E731
                y = m(xr)
            else:
                f = lambda: torch.nn.functional.layer_norm(x, (hidden,), w, b, 1e-5)  # noqa: E731
                y = torch.nn.functional.layer_norm(xr, (hidden,), w, b, 1e-5)
            with torch.no_grad():
                t_f = timeit(f)
            t_b = timeit(lambda: torch.autograd.grad(y, (xr, w, b), g, retain_graph=True))
            fb, bb = 2 * x.numel() * 2, 3 * x.numel() * 2
            print(json.dumps({"hidden": hidden, "rows": n1, "impl": impl, "fwd_us": round(t_f, 1),
                              "fwd_GBps": round(fb / t_f / 1e3, 1), "fwd_of_copy": round(fb / t_f / (2 * rows_bytes / t_copy), 3),
                              "bwd_us": round(t_b, 1), "bwd_GBps": round(bb / t_b / 1e3, 1),
                              "bwd_of_copy": round(bb / t_b / (2 * rows_bytes / t_copy), 3)}), flush=True)


if __name__ == "__main__":
    main()
