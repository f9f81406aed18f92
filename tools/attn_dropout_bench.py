#!/usr/bin/env python3
"""Attention with dropout at the GPT-2 medium / BERT-large shapes (d = 64) and d = 128: forward and
forward+backward time with dropout 0.1 vs without, same process.  One JSON line per (shape, arm).

Measured r02 (profiles/attn_dropout_saved_mask_ab_r02.jsonl): a variant that saved the forward's
keep decisions as a bitmask for the backward (instead of regenerating the counter hash) was
SLOWER (fwd +19 %, bwd +4 % at b16 s1024 h16 d64 causal) -- the backward is not hash-bound, and
the extra live registers deepened the spills of the dropout kernel variants -- so it was not kept.  What did pay: a dropout-only kernel variant (MODE 1, bias code compiled
out): the d=64 forward drops from 256 VGPRs + 56 spilled to 188 with no spills, fwd 0.177 -> 0.134
ms and fwd+bwd 0.718 -> 0.622 ms at b16 s1024 h16 d64 causal (profiles/attn_dropout_modes_r02.jsonl)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from apex.ops.attention import flash_attn_func  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    for (b, s, h, d, causal) in [(16, 1024, 16, 64, True), (32, 512, 16, 64, False), (8, 2048, 16, 128, True)]:
        q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
        g = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
        fwd = lambda: flash_attn_func(q, k, v, dropout_p=0.1, causal=causal, seed=1, offset=2)  # noqa: E731

        def fb():
            o = fwd()
            o.backward(g)
        t_f = timeit(lambda: fwd())
        t_fb = timeit(fb)
        print(json.dumps({"b": b, "s": s, "h": h, "d": d, "causal": causal, "p": 0.1, "fwd_ms": round(t_f, 4),
                          "fwd_bwd_ms": round(t_fb, 4), "bwd_ms": round(t_fb - t_f, 4)}), flush=True)
        plain = timeit(lambda: flash_attn_func(q, k, v, causal=causal).backward(g))
        print(json.dumps({"b": b, "s": s, "h": h, "d": d, "causal": causal, "p": 0.0, "fwd_bwd_ms": round(plain, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
