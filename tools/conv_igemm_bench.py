#!/usr/bin/env python3
"""ResNet-50 convolutions (bs 256, bf16, channels_last): MIOpen vs the gfx950 implicit-GEMM tap
kernels (apex.ops.conv) for forward, data gradient and weight gradient; one JSON line per shape
with both times and the max error of the native result vs MIOpen's.  GPU box:
python tools/conv_igemm_bench.py [--batch 256] [--only 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import apex  # noqa: E402,F401
from apex.ops import conv as C  # noqa: E402

from conv_shapes_bench import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", type=int, default=0, help="kernel size filter (0 = all eligible)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    B = a.batch
    tot = {}
    for cin, cout, k, st, h, cnt in SHAPES:
        if cin % 64 or (a.only and k != a.only):
            continue
        pad = k // 2
        ho = (h + 2 * pad - k) // st + 1
        x = torch.randn(B, cin, h, h, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last)
        gy = torch.randn(B, cout, ho, ho, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        args = ([st, st], [pad, pad], [1, 1], False, [0, 0], 1)
        r = {"cin": cin, "cout": cout, "k": k, "stride": st, "h": h, "count": cnt}
        m_f = timeit(lambda: F.conv2d(x, w, None, st, pad))
        n_f = timeit(lambda: C.conv_tap_forward(x, w, st, pad))
        m_d = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, *args, [True, False, False]))
        n_d = timeit(lambda: C.conv_tap_dgrad(gy, w, x.shape, st, pad))
        m_w = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, *args, [False, True, False]))
        n_w = timeit(lambda: C.conv_tap_wgrad(gy, x, w.shape, st, pad, torch.bfloat16))
        yf = F.conv2d(x, w, None, st, pad).float()
        e_f = float((C.conv_tap_forward(x, w, st, pad).float() - yf).abs().max()) / max(1.0, float(yf.abs().max()))
        dx_m, dw_m, _ = torch.ops.aten.convolution_backward(gy, x, w, None, *args, [True, True, False])
        e_d = float((C.conv_tap_dgrad(gy, w, x.shape, st, pad).float() - dx_m.float()).abs().max()) / max(
            1.0, float(dx_m.float().abs().max()))
        dwn = C.conv_tap_wgrad(gy, x, w.shape, st, pad, torch.float32)
        e_w = float((dwn - dw_m.float()).abs().max()) / max(1.0, float(dw_m.float().abs().max()))
        flops = 2.0 * B * ho * ho * cout * cin * k * k
        for key, mt, nt in (("fwd", m_f, n_f), ("dgrad", m_d, n_d), ("wgrad", m_w, n_w)):
            r[f"miopen_{key}_us"] = round(mt * 1e6, 1)
            r[f"native_{key}_us"] = round(nt * 1e6, 1)
            r[f"native_{key}_tflops"] = round(flops / nt / 1e12, 1)
            r[f"speedup_{key}"] = round(mt / nt, 3)
            tot.setdefault(f"miopen_{key}", 0.0)
            tot.setdefault(f"native_{key}", 0.0)
            tot[f"miopen_{key}"] += cnt * mt * 1e3
            tot[f"native_{key}"] += cnt * nt * 1e3
        r["rel_err"] = [round(e_f, 5), round(e_d, 5), round(e_w, 5)]
        print(json.dumps(r), flush=True)
        del x, w, gy
    print(json.dumps({"total_ms_weighted": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
