#!/usr/bin/env python3
"""Host-side cost of one training step of ``bench.py`` (any of its models / flags).

Builds the bench step exactly as ``bench.py`` does (its ``timed`` is swapped for the probe), then

1. times the host enqueue of K steps while the GPU is kept busy by a long spin kernel, so the host
   can never be throttled by the device: a step whose enqueue time includes the spin is blocked on
   a host<->device sync (the cProfile of that step names the call);
2. times K steps the normal way (host enqueue per step vs device time per step from events).

If host enqueue >= device time per step the eager step is host-bound and the trace shows idle
gaps wherever the host falls behind (VERDICT r03 "host idle 1.2 ms/step").

Usage: python tools/host_probe.py [bench.py args...]   (prints one JSON line + a cProfile top list)
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def probe(args, step, dev, world, rank, distributed, B, impl, desc=None):
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    k = max(3, min(args.steps, 10))
    # 1. GPU held busy: host enqueue cost only (or a sync, which shows as ~spin time)
    spin_ms = 400.0
    torch.cuda._sleep(int(spin_ms * 1e-3 * 2.1e9))  # cycles at ~2.1 GHz
    t_launch = time.perf_counter()
    free_host = []
    profs = []
    for i in range(k):
        prof = cProfile.Profile()
        t0 = time.perf_counter()
        prof.enable()
        step()
        prof.disable()
        profs.append(prof)
        free_host.append((time.perf_counter() - t0) * 1e3)
    # the profile of the slowest (blocked) step names the blocking call
    prof = profs[max(range(k), key=lambda i: free_host[i])]
    t_enq = (time.perf_counter() - t_launch) * 1e3
    torch.cuda.synchronize()
    t_total = (time.perf_counter() - t_launch) * 1e3
    # 2. normal eager stepping: host per step vs device per step
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
    host = []
    torch.cuda.synchronize()
    evs[0].record()
    for i in range(k):
        t0 = time.perf_counter()
        step()
        evs[i + 1].record()
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    dev_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(k)]
    res = {
        "free_host_ms_per_step": [round(x, 2) for x in free_host],
        "free_enqueue_total_ms": round(t_enq, 1),
        "free_total_ms_incl_spin": round(t_total, 1),
        "spin_ms": spin_ms,
        "blocked": bool(max(free_host) > 0.5 * spin_ms),
        "eager_host_ms_per_step": [round(x, 2) for x in host],
        "eager_device_ms_per_step": [round(x, 2) for x in dev_ms],
    }
    print(json.dumps(res), flush=True)
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    bench.timed = probe
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
    bench.main()
