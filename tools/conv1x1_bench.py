#!/usr/bin/env python3
"""ResNet-50 (bs 256, bf16, channels_last) 1x1 stride-1 convolutions: MIOpen (nn.Conv2d) vs the
same convolution as a GEMM on the NHWC [N*H*W, C] view (hipBLASLt), fwd and fwd+bwd.
Prints one JSON line per shape.  Run on the GPU box: python tools/conv1x1_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


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


def gemm_conv(x, w):
    n, c, h, wd = x.shape
    x2 = x.permute(0, 2, 3, 1).reshape(-1, c)
    y2 = torch.matmul(x2, w.view(w.size(0), c).t())
    return y2.view(n, h, wd, -1).permute(0, 3, 1, 2)


def main():
    torch.backends.cudnn.benchmark = True
    shapes = [(64, 64, 56), (64, 256, 56), (256, 64, 56), (256, 128, 56), (128, 512, 28), (512, 128, 28),
              (512, 256, 28), (256, 1024, 14), (1024, 256, 14), (1024, 512, 14), (512, 2048, 7), (2048, 512, 7)]
    for cin, cout, hw in shapes:
        x = torch.randn(256, cin, hw, hw, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        conv = torch.nn.Conv2d(cin, cout, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        gy = torch.randn(256, cout, hw, hw, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        t_m_f = timeit(lambda: conv(x))
        t_g_f = timeit(lambda: gemm_conv(x, conv.weight))
        y = conv(x)
        t_m_b = timeit(lambda: torch.autograd.grad(y, (x, conv.weight), gy, retain_graph=True))
        yg = gemm_conv(x, conv.weight)
        t_g_b = timeit(lambda: torch.autograd.grad(yg, (x, conv.weight), gy, retain_graph=True))
        assert yg.is_contiguous(memory_format=torch.channels_last)
        fl = 2.0 * 256 * hw * hw * cin * cout
        err = (yg.float() - y.float()).abs().max().item()
        extra = {}
        try:
            import apex
            G = apex._native._C.gemm
            x2 = x.detach().permute(0, 2, 3, 1).reshape(-1, cin)
            w2 = conv.weight.detach().view(cout, cin).contiguous()
            gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
            t_a_f = timeit(lambda: G.linear(x2, w2, None, 0, False))
            t_a_b = timeit(lambda: (G.linear_dgrad(gy2, w2, 0, None), G.linear_wgrad(gy2, x2)))
            ya = G.linear(x2, w2, None, 0, False)[0].view(256, hw, hw, cout).permute(0, 3, 1, 2)
            extra = dict(apex_fwd_ms=t_a_f, apex_bwd_ms=t_a_b, apex_fwd_speedup=t_m_f / t_a_f,
                         apex_bwd_speedup=t_m_b / t_a_b, apex_err=(ya.float() - y.float()).abs().max().item(),
                         apex_fwd_tflops=fl / t_a_f / 1e9)
        except Exception as e:  # noqa: BLE001
            extra = dict(apex_error=repr(e)[:200])
        print(json.dumps(dict(cin=cin, cout=cout, hw=hw, miopen_fwd_ms=t_m_f, gemm_fwd_ms=t_g_f, miopen_bwd_ms=t_m_b,
                              gemm_bwd_ms=t_g_b, fwd_speedup=t_m_f / t_g_f, bwd_speedup=t_m_b / t_g_b,
                              gemm_fwd_tflops=fl / t_g_f / 1e9, max_abs_err=err, **extra)), flush=True)


if __name__ == "__main__":
    main()
