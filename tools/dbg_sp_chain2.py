#!/usr/bin/env python3
"""Debug: record every conv_tap_forward call (input, output, statistics partials) of the linked
and the unlinked chain forward and compare them call by call."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402


def main():
    import apex  # noqa: F401
    from apex.models.resnet import run_linked
    from apex.ops import bottleneck_bn
    from apex.ops import conv as convops
    import test_bottleneck_block as T

    torch.manual_seed(3)
    a = T._chain().cuda().to(memory_format=torch.channels_last).train()
    xc = torch.randn(4, 64, 14, 14, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
    rec = []
    orig = convops.conv_tap_forward

    def spy(x, w, stride, pad, stats_shift=None):
        sh = None if stats_shift is None else stats_shift.clone()
        r = orig(x, w, stride, pad, stats_shift=stats_shift)
        y, part = (r, None) if stats_shift is None else r
        rec.append((x.clone(), w.clone(), sh, y.clone(), None if part is None else part.clone()))
        return r

    convops.conv_tap_forward = spy
    outs = []
    fwd0 = bottleneck_bn._BottleneckFn.forward

    def fwd_spy(ctx, *args):
        o = fwd0(ctx, *args)
        outs.append(o)  # deferred outputs are filled later: compared after the whole walk
        return o

    bottleneck_bn._BottleneckFn.forward = staticmethod(fwd_spy)
    bottleneck_bn._ENABLED, bottleneck_bn.FORCE_NATIVE = True, True
    runs = {}
    for name, linked in (("L1", True), ("L2", True), ("U1", False), ("U2", False)):
        rec.clear()
        outs.clear()
        m = copy.deepcopy(a)
        xi = xc.clone().requires_grad_(True)
        if linked:
            y = run_linked(list(m), xi)
        else:
            y = xi
            for blk in m:
                y = blk(y)
        y = y[0] if isinstance(y, tuple) else y
        torch.cuda.synchronize()
        runs[name] = (y.detach().clone(), list(rec), [o.detach().clone() for o in outs])
    for p, q in (("L1", "L2"), ("U1", "U2"), ("L1", "U1")):
        ya, ra, oa = runs[p]
        yb, rb, ob = runs[q]
        print(p, q, "final equal", torch.equal(ya, yb), "calls", len(ra), len(rb))
        for k, (u, v) in enumerate(zip(oa, ob)):
            d = (u.float() - v.float()).abs()
            print("  block", k, "out equal", torch.equal(u, v), "ndiff", int((u != v).sum()), "max", float(d.max()))
        for k, (ca, cb) in enumerate(zip(ra, rb)):
            print("  call", k, "x", torch.equal(ca[0], cb[0]), "w", torch.equal(ca[1], cb[1]),
                  "shift", None if ca[2] is None else torch.equal(ca[2], cb[2]),
                  "y", torch.equal(ca[3], cb[3]), "part", None if ca[4] is None else torch.equal(ca[4], cb[4]),
                  "xshape", tuple(ca[0].shape), tuple(ca[0].stride()), ca[0].data_ptr() % 256)


if __name__ == "__main__":
    main()
