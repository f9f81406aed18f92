#!/usr/bin/env python3
"""The MLP's GeLU on the GEMM: library GEMM + a separate GeLU pass vs the native MFMA GEMM with the
GeLU(-aux) epilogue, forward (fc1) and backward (fc2's data gradient with the dGeLU epilogue + the
bias-gradient column sum), at the GPT-2 medium / BERT-large MLP shape (16384 tokens, 1024 -> 4096
-> 1024, bf16).  One JSON line per (op, route).  Run on the GPU box."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timeit(fn, iters=30, warmup=5):
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

    g = _native.require("gemm").gemm
    lt = _native.require("lt_gemm").lt_gemm
    dt = torch.bfloat16
    torch.manual_seed(0)
    for m, h, f in [(16384, 1024, 4096), (8192, 1024, 4096), (16384, 768, 3072)]:
        x = torch.randn(m, h, device="cuda", dtype=dt)
        w1 = torch.randn(f, h, device="cuda", dtype=dt) * 0.03
        b1 = torch.randn(f, device="cuda", dtype=dt) * 0.1
        w2 = torch.randn(h, f, device="cuda", dtype=dt) * 0.03
        gy = torch.randn(m, h, device="cuda", dtype=dt)
        z = lt.linear(x, w1, b1, lt.EPI_BIAS)[0]
        rows = {
            "fwd_lt_bias+gelu_pass": lambda: g.gelu(lt.linear(x, w1, b1, lt.EPI_BIAS)[0]),
            "fwd_native_gelu_aux_epilogue": lambda: g.linear(x, w1, b1, g.EPI_GELU, True),
            "bwd_lt_dgrad+dgelu_colsum_pass": lambda: g.dgelu_column_sum(lt.mm(gy, w2, False, False)[0], z),
            "bwd_torch_dgrad+dgelu_colsum_pass": lambda: g.dgelu_column_sum(gy.matmul(w2), z),
            "bwd_native_dgelu_epilogue+colsum": lambda: _native.column_sum(g.linear_dgrad(gy, w2, g.EPI_DGELU, z), dt),
            "bwd_native_dgelu_epilogue_only": lambda: g.linear_dgrad(gy, w2, g.EPI_DGELU, z),
            "bwd_native_dgelu_bgrad_epilogue": lambda: g.linear_dgrad_bgrad(gy, w2, g.EPI_DGELU, z),
            "fwd_lt_bias_only": lambda: lt.linear(x, w1, b1, lt.EPI_BIAS),
        }
        # numerics of the native epilogue forms against the unfused composition
        y_ref = torch.nn.functional.gelu(z.float(), approximate="tanh")
        y_nat, aux = g.linear(x, w1, b1, g.EPI_GELU, True)
        dh = gy.float() @ w2.float()
        t = torch.tanh(0.7978845608 * (z.float() + 0.044715 * z.float() ** 3))
        dgelu = 0.5 * (1 + t) + 0.5 * z.float() * (1 - t * t) * 0.7978845608 * (1 + 3 * 0.044715 * z.float() ** 2)
        gz_ref = dh * dgelu
        gz_nat = g.linear_dgrad(gy, w2, g.EPI_DGELU, z)
        err = {"fwd_rel": float((y_nat.float() - y_ref).norm() / y_ref.norm()),
               "aux_rel": float((aux.float() - z.float()).norm() / z.float().norm()),
               "bwd_rel": float((gz_nat.float() - gz_ref).norm() / gz_ref.norm())}
        print(json.dumps({"m": m, "h": h, "f": f, **{k: round(v, 5) for k, v in err.items()}}), flush=True)
        for name, fn in rows.items():
            us = timeit(fn)
            print(json.dumps({"m": m, "h": h, "f": f, "route": name, "us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
