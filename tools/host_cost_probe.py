#!/usr/bin/env python3
"""Host-side cost of the runtime calls the ResNet-50 step makes (no tracing): hipGetDeviceCount
(via torch._C._cuda_getDeviceCount), a hipBLASLt GEMM enqueue (apex lt_gemm.mm, the stage-3/4
1x1 route) and a native fused-1x1 enqueue, each timed over many calls without a device sync."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def host_us(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return dt


def main():
    import apex

    torch.cuda.init()
    print("hipGetDeviceCount us:", round(host_us(torch._C._cuda_getDeviceCount, 1000), 2), flush=True)
    lt = apex._native.require("lt_gemm").lt_gemm
    conv = apex._native.require("conv").conv
    a = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(256, 1024, device="cuda", dtype=torch.bfloat16)
    print("lt.mm enqueue us:", round(host_us(lambda: lt.mm(a, w, False, True)), 2), flush=True)
    print("torch.matmul enqueue us:", round(host_us(lambda: torch.matmul(a, w.t())), 2), flush=True)
    x = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16)
    w1 = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
    print("native bn1x1 enqueue us:", round(host_us(lambda: conv.bn1x1(x, w1, False, None, None, True)), 2), flush=True)
    y = torch.empty_like(a)
    print("torch copy_ enqueue us:", round(host_us(lambda: y.copy_(a)), 2), flush=True)


if __name__ == "__main__":
    main()
