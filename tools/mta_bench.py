#!/usr/bin/env python3
"""Bandwidth of the multi-tensor ops (one JSON line per case): FusedAdam fused-amp step
(bf16 grads, fp32 master/m/v, bf16 model copy = 28 B/param), fp32 Adam (32 B/param), SGD,
scale and L2 norm, over 24 x 4M-element tensors.  Run once per native variant
(APEX_AMD_NATIVE_SO=rocm-apex_amd/_variants/_C_<v>.so) to A/B engine changes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from apex import _native, amp_C  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    assert _native.available(), _native.import_error
    variant = os.path.basename(os.environ.get("APEX_AMD_NATIVE_SO", "default"))
    n, t = 4 * 1024 * 1024, 24
    dev = "cuda"
    P = [torch.randn(n, device=dev) for _ in range(t)]
    M = [torch.zeros(n, device=dev) for _ in range(t)]
    V = [torch.zeros(n, device=dev) for _ in range(t)]
    G16 = [torch.randn(n, device=dev, dtype=torch.bfloat16) for _ in range(t)]
    O16 = [torch.empty(n, device=dev, dtype=torch.bfloat16) for _ in range(t)]
    G32 = [torch.randn(n, device=dev) for _ in range(t)]
    noop = torch.zeros(1, dtype=torch.int32, device=dev)
    lr = torch.tensor([1e-4], device=dev)
    step = torch.tensor([1.0], device=dev)
    inv = torch.tensor([1.0], device=dev)
    elems = n * t
    cases = {
        "adam_fused_amp_bf16": (lambda: amp_C.multi_tensor_adam_capturable(
            65536, noop, [G16, P, M, V, O16], lr, 0.9, 0.999, 1e-8, step, 1, 1, 0.0, inv), 28),
        "adam_fp32": (lambda: amp_C.multi_tensor_adam(65536, noop, [G32, P, M, V], 1e-4, 0.9, 0.999, 1e-8, 1, 1, 1,
                                                      0.0), 28),
        "adam_fp32_chunk16k": (lambda: amp_C.multi_tensor_adam(16384, noop, [G32, P, M, V], 1e-4, 0.9, 0.999, 1e-8, 1, 1,
                                                                1, 0.0), 28),
        "adam_fp32_chunk256k": (lambda: amp_C.multi_tensor_adam(262144, noop, [G32, P, M, V], 1e-4, 0.9, 0.999, 1e-8, 1,
                                                                 1, 1, 0.0), 28),
        "sgd_fp32_mom": (lambda: amp_C.multi_tensor_sgd(65536, noop, [G32, P, M], 0.0, 0.9, 0.0, 1e-4, False, False,
                                                        False, 1.0), 20),
        "sgd_fp32_mom_chunk16k": (lambda: amp_C.multi_tensor_sgd(16384, noop, [G32, P, M], 0.0, 0.9, 0.0, 1e-4, False,
                                                                 False, False, 1.0), 20),
        "scale_bf16_to_fp32": (lambda: amp_C.multi_tensor_scale(65536, noop, [G16, V], 0.5), 6),
        "l2norm_fp32": (lambda: amp_C.multi_tensor_l2norm(65536, noop, [G32], False), 4),
    }
    # the in-run roof: an elementwise kernel (torch.mul by 1) moving the fp32 Adam step's bytes
    # (half read, half written), timed the same way in the same process
    src = torch.empty(elems * 28 // 8, device=dev).uniform_()
    dst = torch.empty_like(src)
    roof = elems * 28 / timeit(lambda: torch.mul(src, 1.0, out=dst)) / 1e9
    del src, dst
    print(json.dumps({"variant": variant, "case": "copy_roof_28B", "GBps": round(roof, 1)}), flush=True)
    for name, (fn, bpe) in cases.items():
        sec = timeit(fn)
        gbps = elems * bpe / sec / 1e9
        print(json.dumps({"variant": variant, "case": name, "us": round(sec * 1e6, 1), "GBps": round(gbps, 1),
                          "bytes_per_elem": bpe, "pct_of_copy": round(100 * gbps / roof, 1)}), flush=True)


if __name__ == "__main__":
    main()
