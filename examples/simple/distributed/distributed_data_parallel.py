#!/usr/bin/env python3
"""Minimal amp + apex DDP loop (reference examples/simple/distributed/distributed_data_parallel.py).

``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
examples/simple/distributed/distributed_data_parallel.py`` (RCCL on GPUs; ``--cpu`` runs over
gloo for a quick check without a GPU)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import torch  # noqa: E402

from apex import amp  # noqa: E402
from apex.parallel import DistributedDataParallel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--steps", type=int, default=500)
    a = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and not a.cpu
    if use_gpu:
        torch.cuda.set_device(local)
    torch.distributed.init_process_group(backend="nccl" if use_gpu else "gloo", init_method="env://")
    dev = torch.device("cuda") if use_gpu else torch.device("cpu")
    torch.manual_seed(torch.distributed.get_rank())
    N, D_in, D_out = 64, 1024, 16
    x = torch.randn(N, D_in, device=dev)
    y = torch.randn(N, D_out, device=dev)
    model = torch.nn.Linear(D_in, D_out).to(dev)
    optimizer = torch.optim.SGD(model.parameters(), lr=1e-3)
    if use_gpu:
        model, optimizer = amp.initialize(model, optimizer, opt_level="O1")
    model = DistributedDataParallel(model)
    loss_fn = torch.nn.MSELoss()
    for t in range(a.steps):
        optimizer.zero_grad()
        loss = loss_fn(model(x), y)
        if use_gpu:
            with amp.scale_loss(loss, optimizer) as scaled:
                scaled.backward()
        else:
            loss.backward()
        optimizer.step()
    if torch.distributed.get_rank() == 0:
        print("final loss = ", loss.item())


if __name__ == "__main__":
    main()
