#!/usr/bin/env python3
"""Which part of the ResNet-50 amp training step breaks hipGraph capture?  Captures growing
prefixes of the step (each in a fresh graph, after side-stream warm-up) and reports the first
failure with its traceback."""
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from apex import amp
    from apex.models import resnet50
    from apex.optimizers import FusedAdam

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B = int(os.environ.get("PROBE_BATCH", "64"))
    model = resnet50().to(dev).to(memory_format=torch.channels_last)
    opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=1e-4,
                    materialize_master_grads=os.environ.get("PROBE_MATERIALIZE", "0") == "1")
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16,
                                keep_batchnorm_fp32=True, verbosity=0)
    crit = torch.nn.CrossEntropyLoss()
    x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)

    def fwd():
        return crit(model(x), y)

    def fwd_bwd_plain():
        loss = fwd()
        loss.backward()
        return loss

    def amp_bwd():
        loss = fwd()
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        return loss

    def full():
        loss = amp_bwd()
        opt.step()
        return loss

    s = torch.cuda.Stream()
    for name, fn in (("forward", fwd), ("forward+backward", fwd_bwd_plain), ("amp scale_loss+backward", amp_bwd),
                     ("full step", full)):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                fn()
            g.replay()
            torch.cuda.synchronize()
            print(f"[probe] {name}: capture + replay OK", flush=True)
        except Exception:
            print(f"[probe] {name}: FAILED", flush=True)
            traceback.print_exc()
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
