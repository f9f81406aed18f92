#!/usr/bin/env python3
"""Debug: spatial-tile 3x3 kernel determinism and the linked-vs-unlinked chain forward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import copy  # noqa: E402

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    import apex  # noqa: F401
    from apex.ops import conv as C
    import test_bottleneck_block as T

    torch.manual_seed(0)
    x = torch.randn(4, 64, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    sh = torch.randn(64, device="cuda") * 0.1
    ext = C._conv_ext()
    outs = []
    for cfg in (21, 21, 7, 7):
        ext.force_fprop_cfg(cfg)
        y, part = C.conv_tap_forward(x, w, 1, 1, stats_shift=sh)
        outs.append((y.clone(), part.clone()))
    ext.force_fprop_cfg(-1)
    print("sp det y", torch.equal(outs[0][0], outs[1][0]), "part", torch.equal(outs[0][1], outs[1][1]))
    print("sp vs cfg7 y maxdiff", float((outs[0][0].float() - outs[2][0].float()).abs().max()))
    yr = F.conv2d(x.float(), w.float(), None, 1, 1)
    print("sp vs fp32", float((outs[0][0].float() - yr).abs().max()), "cfg7 vs fp32", float((outs[2][0].float() - yr).abs().max()))
    torch.manual_seed(3)
    a = T._chain().cuda().to(memory_format=torch.channels_last).train()
    b = copy.deepcopy(a)
    xc = torch.randn(4, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    # forward only, no backward, both walks
    from apex.models.resnet import run_linked
    from apex.ops import bottleneck_bn
    old = bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE
    bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE = True, True
    a2, b2 = copy.deepcopy(a), copy.deepcopy(a)
    with torch.no_grad():
        pass
    y1 = run_linked(list(a2), xc.clone().requires_grad_(True))
    y1 = y1[0] if isinstance(y1, tuple) else y1
    y1c = y1.detach().clone()
    y2 = xc.clone().requires_grad_(True)
    for blk in b2:
        y2 = blk(y2)
    print("fwd-only linked vs unlinked equal", torch.equal(y1.detach(), y2.detach()),
          float((y1.detach().float() - y2.detach().float()).abs().max()))
    y1.backward(gy)
    print("linked y unchanged by backward", torch.equal(y1.detach(), y1c))
    bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE = old
    ya, ga, pa, ca = T._run_chain(a, xc, gy, True)
    yb, gb, pb, cb = T._run_chain(b, xc, gy, True, linked=False)
    print("calls", ca, cb)
    print("chain y equal", torch.equal(ya, yb), "maxdiff", float((ya.float() - yb.float()).abs().max()),
          "count", int((ya != yb).sum()), "of", ya.numel())


if __name__ == "__main__":
    main()
