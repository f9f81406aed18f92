#!/usr/bin/env python3
"""ResNet-50 stem at bs 256 (224x224, bf16, channels_last): the native stem node (ops/stem.py)
against the module path (channel-padded library conv + fused NHWC BN/ReLU/pool), forward and
forward+backward, plus each native kernel on its own.  One JSON line per row.
Run on the GPU box: python tools/stem_node_bench.py [--batch 256]"""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    import apex  # noqa: F401
    from apex import _native
    from apex.contrib.groupbn import bn_relu_maxpool
    from apex.models.resnet import resnet50
    from apex.ops import stem

    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    dt = torch.bfloat16
    model = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    model.conv1.to(dt)
    ref = copy.deepcopy(model)
    x = torch.randn(args.batch, 3, 224, 224, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    gout = torch.randn(args.batch, 64, 56, 56, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)

    def nat_f():
        return stem.stem_forward(model.conv1, model.bn1, model.maxpool, x)

    def mod_f():
        return bn_relu_maxpool(ref.conv1(x), ref.bn1, ref.maxpool)

    def nat_fb():
        nat_f().backward(gout)

    def mod_fb():
        mod_f().backward(gout)

    rows = []
    with torch.no_grad():
        rows.append(("native_fwd", timeit(nat_f)))
        rows.append(("module_fwd", timeit(mod_f)))
    rows.append(("native_fwd_bwd", timeit(nat_fb)))
    rows.append(("module_fwd_bwd", timeit(mod_fb)))

    ext = _native.require("conv").conv
    bn = model.bn1
    y, part, xp = ext.stem_fprop(x, model.conv1.weight, bn.running_mean)
    m = float(y.size(0) * y.size(2) * y.size(3))
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    sm, si, coef = ext.bn_finalize(part, m, rm, bn.weight, bn.bias, rm, rv, 1e-5, 0.1)
    p, idx = ext.stem_pool(y, coef)
    part2 = ext.stem_reduce(gout, idx, y, coef, sm)
    cb, gg, gb = ext.bnbwd_finalize(part2, m, sm, si, bn.weight)
    rows.append(("k_fprop(pad+pack+conv+stats)", timeit(lambda: ext.stem_fprop(x, model.conv1.weight, bn.running_mean))))
    rows.append(("k_pool_fwd", timeit(lambda: ext.stem_pool(y, coef))))
    rows.append(("k_bwd_reduce", timeit(lambda: ext.stem_reduce(gout, idx, y, coef, sm))))
    rows.append(("k_wgrad(+reduce)", timeit(lambda: ext.stem_wgrad(gout, idx, y, coef, cb.view(-1), xp,
                                                                   model.conv1.weight))))
    for name, us in rows:
        print(json.dumps({"row": name, "us": round(us, 1), "batch": args.batch}))


if __name__ == "__main__":
    main()
