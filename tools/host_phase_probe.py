"""Host time per phase of the ResNet-50 bench step (forward / loss / zero_grad / backward /
optimizer) against the device time of the same phases, steady state, no device sync inside the
timed steps: tells whether the host is ahead of the GPU or blocked somewhere in a phase (a phase
whose host time tracks its device time while the host should be steps ahead is blocking).

    python tools/host_phase_probe.py [--steps 12] [--warmup 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--sync-debug", action="store_true")
    args = ap.parse_args()
    import apex
    from apex import amp
    from apex.models import resnet50
    from apex.optimizers import FusedAdam

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = resnet50(fused_bn=True).to(dev).to(memory_format=torch.channels_last)
    opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=1e-4, materialize_master_grads=False)  # as bench.py
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16,
                                keep_batchnorm_fp32=True, verbosity=0)
    crit = torch.nn.CrossEntropyLoss().to(dev)
    images = torch.randn(256, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    target = torch.randint(0, 1000, (256,), device=dev)
    names = ["forward", "loss", "zero_grad", "backward", "amp_exit", "optimizer"]

    def step(rec):
        ts = [time.perf_counter()]
        evs = []

        def mark():
            ts.append(time.perf_counter())
            if rec:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                evs.append(e)

        if rec:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
        out = model(images)
        mark()
        loss = crit(out, target)
        mark()
        opt.zero_grad()
        mark()
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
            mark()
        mark()
        opt.step()
        mark()
        return ts, evs

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if args.sync_debug:
        # one step with torch's synchronizing-op detector: each blocking call prints its stack
        import traceback
        import warnings

        def show(msg, cat, fn, ln, file=None, line=None):
            print(f"[sync] {msg}", file=sys.stderr)
            traceback.print_stack(limit=14, file=sys.stderr)

        warnings.showwarning = show
        warnings.simplefilter("always")
        torch.cuda.set_sync_debug_mode("warn")
        step(False)
        torch.cuda.set_sync_debug_mode("default")
        torch.cuda.synchronize()
    rows = [step(True) for _ in range(args.steps)]
    torch.cuda.synchronize()
    for i, (ts, evs) in enumerate(rows):
        host = {n: round(1e3 * (ts[j + 1] - ts[j]), 3) for j, n in enumerate(names)}
        gpu = {n: round(evs[j].elapsed_time(evs[j + 1]), 3) for j, n in enumerate(names)}
        lead = round(1e3 * (ts[0] - rows[0][0][0]), 3)
        print(json.dumps({"step": i, "host_ms": host, "gpu_ms": gpu, "host_t0_ms": lead,
                          "host_total": round(sum(host.values()), 3), "gpu_total": round(sum(gpu.values()), 3)}),
              flush=True)


if __name__ == "__main__":
    main()
