#!/usr/bin/env python3
"""Attention fwd+bwd loop for rocprofv3 per-kernel timing (both backward variants).
Run: rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o attn -- python3 tools/attn_prof.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from apex.ops.attention import flash_attn_func  # noqa: E402


def main():
    for (b, s, h, d, causal) in [(8, 2048, 16, 128, True), (8, 2048, 16, 128, False), (16, 1024, 16, 64, False)]:
        q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn_like(q, requires_grad=True)
        v = torch.randn_like(q, requires_grad=True)
        for mode in ("split", "atomic"):
            os.environ["APEX_ATTN_BWD"] = mode
            for _ in range(5):
                o = flash_attn_func(q, k, v, causal=causal)
                torch.autograd.grad(o, (q, k, v), torch.ones_like(o))
        torch.cuda.synchronize()
    print("attn_prof done", flush=True)


if __name__ == "__main__":
    main()
