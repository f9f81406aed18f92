#!/usr/bin/env python3
"""ResNet-50 stem (7x7/2 conv, 64 filters, bs 256, bf16, channels_last) under MIOpen with the
input channel count padded 3 -> 4 / 8 (zero channels, zero weight slices): fwd and fwd+wgrad
times.  One JSON line per variant.  Run on the GPU box: python tools/stem_bench.py"""
import json

import torch
import torch.nn.functional as F


def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    x3 = torch.randn(256, 3, 224, 224, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    w3 = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).to(torch.bfloat16).to(memory_format=torch.channels_last)
    w3.requires_grad_(True)
    gy = torch.randn(256, 64, 112, 112, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref = None
    for cin in (3, 4, 8):
        def fwd():
            x = F.pad(x3, (0, 0, 0, 0, 0, cin - 3)) if cin > 3 else x3
            w = F.pad(w3, (0, 0, 0, 0, 0, cin - 3)) if cin > 3 else w3
            x = x.contiguous(memory_format=torch.channels_last)
            w = w.contiguous(memory_format=torch.channels_last)
            return F.conv2d(x, w, stride=2, padding=3)

        y = fwd()
        t_f = timeit(fwd)

        def fb():
            out = fwd()
            torch.autograd.grad(out, (w3,), gy)

        t_b = timeit(fb)
        gw = torch.autograd.grad(fwd(), (w3,), gy)[0]
        if ref is None:
            ref = (y.float(), gw.float())
        err_y = (y.float() - ref[0]).abs().max().item()
        err_w = ((gw.float() - ref[1]).abs().max() / ref[1].abs().max()).item()
        print(json.dumps(dict(cin=cin, fwd_ms=t_f, fwd_wgrad_ms=t_b, y_cl=y.is_contiguous(memory_format=torch.channels_last),
                              max_err_y=err_y, rel_err_gw=err_w)), flush=True)


if __name__ == "__main__":
    main()
