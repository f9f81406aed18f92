#!/usr/bin/env python3
"""Gradient error of the chained bottleneck nodes AND of the per-module fused path against an
fp32 PyTorch ResNet-50 with the same weights (debug aid for tests/test_bottleneck_block.py):
prints, per parameter group, both paths' relative error vs fp32 and their distance to each
other.  Usage: python tools/dbg_block_chain.py [force] [batch] [size]"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex  # noqa: E402,F401
from apex.models import resnet50  # noqa: E402
from apex.ops import bottleneck_bn  # noqa: E402


def rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def main():
    force = len(sys.argv) > 1 and sys.argv[1] == "force"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 96
    bottleneck_bn.FORCE_NATIVE = force
    torch.manual_seed(0)
    ref = resnet50().cuda()
    m1 = resnet50(fused_bn=True).cuda()
    m1.load_state_dict(ref.state_dict())
    m1 = m1.to(memory_format=torch.channels_last)
    for mod in m1.modules():
        if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear)):
            mod.to(torch.bfloat16)
    m2 = copy.deepcopy(m1)
    x = torch.randn(batch, 3, size, size, device="cuda")
    tgt = torch.randint(0, 1000, (batch,), device="cuda")
    xb = x.to(torch.bfloat16).to(memory_format=torch.channels_last)
    torch.nn.functional.cross_entropy(ref(x), tgt).backward()
    for model, en in ((m1, True), (m2, False)):
        bottleneck_bn._ENABLED = en
        loss = torch.nn.functional.cross_entropy(model(xb).float(), tgt)
        loss.backward()
    g0 = dict(ref.named_parameters())
    g2 = dict(m2.named_parameters())
    rows = []
    for n, p in m1.named_parameters():
        rows.append((rel(p.grad, g0[n].grad), rel(g2[n].grad, g0[n].grad), rel(p.grad, g2[n].grad), n))
    rows.sort(reverse=True)
    print("node_vs_fp32 module_vs_fp32 node_vs_module param")
    for r in rows[:20]:
        print("%.4f %.4f %.4f %s" % r)
    import statistics
    print("median node %.4f module %.4f" % (statistics.median(r[0] for r in rows), statistics.median(r[1] for r in rows)))


if __name__ == "__main__":
    main()
