#!/usr/bin/env python3
"""ImageNet training with apex amp + apex DDP on MI355X (reference examples/imagenet/main_amp.py).

One process per GPU (``python -m torch.distributed.run --nproc-per-node 8 --master-addr
127.0.0.1 examples/imagenet/main_amp.py ...``), RCCL over xGMI.  Features of the reference kept:
opt levels O0-O5, ``--loss-scale``, ``--keep-batchnorm-fp32``, apex ``DistributedDataParallel``
(``--delay-allreduce``), ``--sync_bn`` (apex SyncBatchNorm), channels_last, a data prefetcher
that uploads + normalises the next batch on a side HIP stream, and the "Speed" print
(world * batch / batch_time).  MI355X additions: the fused NHWC BN+ReLU ResNet
(``--bn fused``), FusedAdam / FusedSGD / FusedLAMB, and ``--data synthetic`` (no dataset
needed); ``--data DIR`` reads an ImageFolder when torchvision is importable.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import apex  # noqa: E402
from apex import amp  # noqa: E402
from apex.models import resnet as resnet_mod  # noqa: E402
from apex.optimizers import FusedAdam, FusedLAMB, FusedSGD  # noqa: E402


def parse():
    p = argparse.ArgumentParser(description="PyTorch ImageNet training (apex / MI355X)")
    p.add_argument("--data", default="synthetic")
    p.add_argument("--arch", "-a", default="resnet50")
    p.add_argument("--epochs", default=1, type=int)
    p.add_argument("--iters-per-epoch", default=100, type=int, help="synthetic data: steps per epoch")
    p.add_argument("-b", "--batch-size", default=256, type=int, help="per-process batch")
    p.add_argument("--lr", default=0.1, type=float)
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--weight-decay", "--wd", default=1e-4, type=float)
    p.add_argument("--optimizer", default="sgd", choices=["sgd", "adam", "lamb"])
    p.add_argument("--print-freq", "-p", default=10, type=int)
    p.add_argument("--opt-level", default="O2")
    p.add_argument("--keep-batchnorm-fp32", default=None)
    p.add_argument("--loss-scale", default=None)
    p.add_argument("--channels-last", default=True, type=lambda s: s.lower() not in ("0", "false", "no"))
    p.add_argument("--sync_bn", action="store_true")
    p.add_argument("--bn", default="fused", choices=["fused", "torch"])
    p.add_argument("--delay-allreduce", action="store_true")
    p.add_argument("--prof", default=-1, type=int, help="stop after this many iterations (profiling)")
    p.add_argument("--workers", default=4, type=int)
    return p.parse_args()


class SyntheticLoader:
    """Host-side uint8 images + labels, like a decoded JPEG batch from a DataLoader."""

    def __init__(self, batch, n):
        self.batch, self.n = batch, n
        g = torch.Generator().manual_seed(0)
        self.images = torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8, generator=g).pin_memory() \
            if torch.cuda.is_available() else torch.randint(0, 256, (batch, 224, 224, 3), dtype=torch.uint8)
        self.labels = torch.randint(0, 1000, (batch,), generator=g)

    def __len__(self):
        return self.n

    def __iter__(self):
        for _ in range(self.n):
            yield self.images, self.labels


class DataPrefetcher:
    """Upload + normalise batch i+1 on a side stream while batch i trains (reference
    main_amp.py:264-318); NHWC uint8 -> channels_last float normalised in one kernel chain."""

    def __init__(self, loader, channels_last):
        self.loader = iter(loader)
        self.stream = torch.cuda.Stream()
        self.mean = torch.tensor([0.485 * 255, 0.456 * 255, 0.406 * 255], device="cuda").view(1, 3, 1, 1)
        self.std = torch.tensor([0.229 * 255, 0.224 * 255, 0.225 * 255], device="cuda").view(1, 3, 1, 1)
        self.mf = torch.channels_last if channels_last else torch.contiguous_format
        self.preload()

    def preload(self):
        try:
            images, labels = next(self.loader)
        except StopIteration:
            self.next_input = self.next_target = None
            return
        with torch.cuda.stream(self.stream):
            x = images.cuda(non_blocking=True).permute(0, 3, 1, 2).float()
            self.next_input = x.sub_(self.mean).div_(self.std).contiguous(memory_format=self.mf)
            self.next_target = labels.cuda(non_blocking=True)

    def next(self):
        torch.cuda.current_stream().wait_stream(self.stream)
        x, y = self.next_input, self.next_target
        if x is not None:
            x.record_stream(torch.cuda.current_stream())
            y.record_stream(torch.cuda.current_stream())
        self.preload()
        return x, y


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    torch.cuda.set_device(local)
    if distributed:
        dist.init_process_group(backend="nccl", init_method="env://")
    torch.backends.cudnn.benchmark = True
    fused_bn = args.bn == "fused" and args.channels_last
    sync = args.sync_bn and distributed
    # fused NHWC BN: --sync_bn shares the statistics over all ranks inside the fused kernels
    # (bn_group = world); torch BN: converted to apex SyncBatchNorm, which detects channels_last
    # memory by itself
    model = getattr(resnet_mod, args.arch)(fused_bn=fused_bn, bn_group=world if (sync and fused_bn) else 1)
    if sync and not fused_bn:
        model = apex.parallel.convert_syncbn_model(model)
    model = model.cuda()
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    lr = args.lr * args.batch_size * world / 256.0
    if args.optimizer == "sgd":
        optimizer = FusedSGD(model.parameters(), lr, momentum=args.momentum, weight_decay=args.weight_decay)
    elif args.optimizer == "adam":
        optimizer = FusedAdam(model.parameters(), lr=lr * 0.01, weight_decay=args.weight_decay)
    else:
        optimizer = FusedLAMB(model.parameters(), lr=lr * 0.01, weight_decay=args.weight_decay)
    model, optimizer = amp.initialize(model, optimizer, opt_level=args.opt_level,
                                      keep_batchnorm_fp32=args.keep_batchnorm_fp32, loss_scale=args.loss_scale,
                                      verbosity=1 if rank == 0 else 0)
    if distributed:
        model = apex.parallel.DistributedDataParallel(model, delay_allreduce=args.delay_allreduce)
    criterion = torch.nn.CrossEntropyLoss().cuda()
    loader = SyntheticLoader(args.batch_size, args.iters_per_epoch)
    for epoch in range(args.epochs):
        model.train()
        pf = DataPrefetcher(loader, args.channels_last)
        x, y = pf.next()
        i = 0
        end = time.time()
        while x is not None:
            i += 1
            if args.prof >= 0 and i > args.prof:
                break
            loss = criterion(model(x), y)
            optimizer.zero_grad()
            with amp.scale_loss(loss, optimizer) as scaled:
                scaled.backward()
            optimizer.step()
            if i % args.print_freq == 0:
                torch.cuda.synchronize()
                bt = (time.time() - end) / args.print_freq
                end = time.time()
                if rank == 0:
                    print("Epoch: [{}][{}/{}]\tTime {:.3f}\tSpeed {:.1f} img/s\tLoss {:.4f}".format(
                        epoch, i, len(loader), bt, world * args.batch_size / bt, loss.item()), flush=True)
            x, y = pf.next()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
