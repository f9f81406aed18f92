#!/usr/bin/env python3
"""Flash-attention kernels for a rocprofv3 counter pass (tools/gpu_pmc_cmd.sh attn tools/pmc_attn.py):
the GPT-2 medium shape (b16 s1024 h16 d64, causal, dropout 0.1), the BERT-large shape (b32 s512 h16
d64, dropout 0.1; again with its additive key-padding bias [b, 1, 1, s], the bench's mode), and d64 /
d128 without dropout (b8 s2048 h16, full), forward + backward, 3 calls
each.  MFMA % of peak in the table is SQ_VALU_MFMA_BUSY_CYCLES over busy cycles."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from apex.ops.attention import flash_attn_func  # noqa: E402


def main():
    torch.manual_seed(0)
    for (b, s, h, d, causal, p, bias) in [(16, 1024, 16, 64, True, 0.1, False), (32, 512, 16, 64, False, 0.1, False),
                                          (32, 512, 16, 64, False, 0.1, True),
                                          (8, 2048, 16, 64, False, 0.0, False), (8, 2048, 16, 128, False, 0.0, False)]:
        q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn_like(q, requires_grad=True)
        v = torch.randn_like(q, requires_grad=True)
        bb = None
        if bias:  # key padding: the last eighth of every sequence masked
            bb = torch.zeros(b, 1, 1, s, device="cuda", dtype=torch.float32)
            bb[..., s - s // 8:] = -10000.0
        for _ in range(3):
            o = flash_attn_func(q, k, v, dropout_p=p, causal=causal, bias=bb)
            torch.autograd.grad(o, (q, k, v), torch.ones_like(o))
        torch.cuda.synchronize()
    print("pmc_attn done", flush=True)


if __name__ == "__main__":
    main()
