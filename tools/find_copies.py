#!/usr/bin/env python3
"""Which torch copies run inside the ResNet-50 headline step: bench.py's step under torch.profiler
(record_shapes + stacks), listing every aten::copy_ / contiguous / to with its device time,
shapes and the innermost repo frames.  Diagnostic only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    captured = {}

    def fake_timed(args, step, dev, world, rank, distributed, B, impl, desc=None):
        captured["step"] = step
        return None

    bench.timed = fake_timed
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
    step = captured["step"]
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    rows = []
    for ev in prof.events():
        if ev.name not in ("aten::copy_", "aten::contiguous", "aten::to", "aten::_to_copy", "aten::clone"):
            continue
        dt = getattr(ev, "device_time_total", None) or getattr(ev, "cuda_time_total", 0)
        if dt < 3:
            continue
        frames = [f for f in (ev.stack or []) if "rocm-apex_amd" in f or "bench.py" in f][:4]
        rows.append((dt, ev.name, ev.input_shapes, frames))
    rows.sort(key=lambda r: -r[0])
    agg = {}
    for dt, name, shapes, frames in rows:
        key = (name, str(shapes))
        n, t, fr = agg.get(key, (0, 0.0, frames))
        agg[key] = (n + 1, t + dt, fr or frames)
    for (name, shapes), (n, t, fr) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"[agg] {n:4d} x {name} {shapes}: {t:9.1f} us", flush=True)
        for f in fr:
            print(f"             {f}", flush=True)
    for dt, name, shapes, frames in rows[:25]:
        print(f"{dt:9.1f} us {name} {shapes}", flush=True)
        for f in frames:
            print(f"             {f}", flush=True)


if __name__ == "__main__":
    main()
