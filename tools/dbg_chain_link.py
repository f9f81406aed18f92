#!/usr/bin/env python3
"""Is the chained-node (BlockLink) gradient error bf16 noise or a hand-off bug?  A 3-block
stage-1 chain in four arms against an fp32 torch reference (nn.BatchNorm2d, same weights):
linked nodes, unlinked nodes (each block called alone), the per-module fused path, and the
linked nodes with the batch doubled (noise shrinks with the batch, a bug does not)."""
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import apex  # noqa: E402,F401
from apex.models.resnet import Bottleneck, conv1x1, run_linked  # noqa: E402
from apex.ops import bottleneck_bn  # noqa: E402


def chain(fused):
    from apex.contrib.groupbn import BatchNorm2d_NHWC

    bn = BatchNorm2d_NHWC(256, fuse_relu=False, torch_channels_last=True) if fused else nn.BatchNorm2d(256)
    ds = nn.Sequential(conv1x1(64, 256, 1, native=fused), bn)
    blocks = [Bottleneck(64, 64, 1, ds, fused_bn=fused), Bottleneck(256, 64, fused_bn=fused),
              Bottleneck(256, 64, fused_bn=fused)]
    if fused:
        for b in blocks[:-1]:
            b.fork_out = True
    return nn.ModuleList(blocks)


def rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def main():
    for batch in (4, 16):
        torch.manual_seed(3)
        ref = chain(False).cuda().float().train()
        for m in ref.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.data.uniform_(0.5, 1.5)
                m.bias.data.uniform_(-0.2, 0.2)
        fused = chain(True).cuda()
        fused.load_state_dict(ref.state_dict())
        for m in fused.modules():
            if isinstance(m, nn.Conv2d):
                m.to(torch.bfloat16)
        fused = fused.to(memory_format=torch.channels_last).train()
        x = torch.randn(batch, 64, 14, 14, device="cuda")
        gy = torch.randn(batch, 256, 14, 14, device="cuda")
        xr = x.clone().requires_grad_(True)
        yr = xr
        for b in ref:
            yr = b(yr)
        yr.backward(gy)
        pr = dict(ref.named_parameters())
        xb = x.to(torch.bfloat16).to(memory_format=torch.channels_last)
        gb = gy.to(torch.bfloat16).to(memory_format=torch.channels_last)
        for arm in ("linked", "unlinked", "module"):
            m = copy.deepcopy(fused)
            old = bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE
            bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE = arm != "module", True
            try:
                xi = xb.clone().requires_grad_(True)
                if arm == "linked":
                    y = run_linked(list(m), xi)
                else:
                    y = xi
                    for b in m:
                        y = b(y)
                y = y[0] if isinstance(y, tuple) else y
                y.backward(gb)
            finally:
                bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE = old
            errs = {n: rel(p.grad, pr[n].grad) for n, p in m.named_parameters()}
            worst = max(errs, key=errs.get)
            print(json.dumps({"batch": batch, "arm": arm, "y": round(rel(y, yr), 4), "dx": round(rel(xi.grad, xr.grad), 4),
                              "median_param": round(sorted(errs.values())[len(errs) // 2], 4),
                              "worst_param": [worst, round(errs[worst], 4)]}), flush=True)


if __name__ == "__main__":
    main()
