#!/usr/bin/env python3
"""A/B sweep of the implicit-GEMM fprop tile configurations (csrc/conv/conv_igemm.hip,
conv_force_fprop_cfg) on the ResNet-50 3x3 shapes (bs 256, bf16): forward and stride-1 data
gradient per configuration, against MIOpen.  One JSON line per (shape, direction)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import apex  # noqa: E402,F401
from apex.ops import conv as C  # noqa: E402
from conv_shapes_bench import SHAPES, timeit  # noqa: E402


def main():
    torch.backends.cudnn.benchmark = True
    ext = C._conv_ext()
    B = int(os.environ.get("BATCH", "256"))
    for cin, cout, k, st, h, cnt in SHAPES:
        if not (k == 3 or (k == 1 and st == 2)) or cin % 64:
            continue
        pad = k // 2
        ho = (h + 2 * pad - k) // st + 1
        x = torch.randn(B, cin, h, h, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last)
        gy = torch.randn(B, cout, ho, ho, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        args = ([st, st], [pad, pad], [1, 1], False, [0, 0], 1)
        ref_f = F.conv2d(x, w, None, st, pad).float()
        r = {"cin": cin, "cout": cout, "stride": st, "h": h, "count": cnt,
             "miopen_fwd_us": round(timeit(lambda: F.conv2d(x, w, None, st, pad)) * 1e6, 1),
             "miopen_dgrad_us": round(timeit(lambda: torch.ops.aten.convolution_backward(
                 gy, x, w, None, *args, [True, False, False])) * 1e6, 1)}
        for cfg in range(21):
            bn = [128, 64, 128, 64, 128, 64, 256, 64, 64, 128, 128, 128, 256, 256, 64, 64, 128, 128, 128, 256, 64][cfg]
            if cout % bn:
                continue
            ext.force_fprop_cfg(cfg)
            y = C.conv_tap_forward(x, w, st, pad).float()
            err = float((y - ref_f).abs().max()) / max(1.0, float(ref_f.abs().max()))
            r[f"cfg{cfg}_fwd_us"] = round(timeit(lambda: C.conv_tap_forward(x, w, st, pad)) * 1e6, 1)
            r[f"cfg{cfg}_dgrad_us"] = round(timeit(lambda: C.conv_tap_dgrad(gy, w, x.shape, st, pad)) * 1e6, 1)
            r[f"cfg{cfg}_err"] = round(err, 4)
        ext.force_fprop_cfg(-1)
        print(json.dumps(r), flush=True)
        del x, w, gy


if __name__ == "__main__":
    main()
