#!/usr/bin/env python3
"""ImageNet training with apex amp + apex DDP on MI355X (reference examples/imagenet/main_amp.py).

Launch: one process per GPU, RCCL over xGMI::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        examples/imagenet/main_amp.py /data/imagenet -a resnet50 -b 256 --opt-level O2

Reference features kept: opt levels O0-O5 with ``--loss-scale`` / ``--keep-batchnorm-fp32``,
apex ``DistributedDataParallel`` (``--delay-allreduce``), ``--sync_bn``, channels_last, a
data prefetcher that uploads and normalises the next batch on a side HIP stream, the
step-decay + 5-epoch-warmup LR schedule, top-1 / top-5 validation reduced over ranks,
``--evaluate``, ``--resume`` from a checkpoint holding model / optimizer / amp state,
``model_best`` tracking, ``--deterministic`` and the "Speed" print (world * batch / time).

MI355X additions: the fused NHWC BN+ReLU ResNet (``--bn fused``, statistics shared over all
ranks inside the fused kernels with ``--sync_bn``), FusedSGD / FusedAdam / FusedLAMB with the
sync-free fused-amp step, and ``synthetic`` data (no dataset needed).  A directory argument
is read as an ImageFolder tree (``train/<class>/*.JPEG``, ``val/<class>/*.JPEG``) decoded with
Pillow in loader workers (torchvision is not required).  Without a GPU the script runs on the
CPU (used by the test suite)."""
import argparse
import math
import os
import random
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import apex  # noqa: E402
from apex import amp  # noqa: E402
from apex.models import resnet as resnet_mod  # noqa: E402
from apex.optimizers import FusedAdam, FusedLAMB, FusedSGD  # noqa: E402

MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)


def parse(argv=None):
    p = argparse.ArgumentParser(description="PyTorch ImageNet training (apex / MI355X)")
    p.add_argument("data", nargs="?", default="synthetic", help="ImageFolder root, or 'synthetic'")
    p.add_argument("--arch", "-a", default="resnet50", choices=["resnet18", "resnet34", "resnet50", "resnet101",
                                                                 "resnet152"])
    p.add_argument("-j", "--workers", default=4, type=int)
    p.add_argument("--epochs", default=90, type=int)
    p.add_argument("--start-epoch", default=0, type=int)
    p.add_argument("--iters-per-epoch", default=100, type=int, help="synthetic data: train steps per epoch")
    p.add_argument("--val-iters", default=10, type=int, help="synthetic data: validation steps")
    p.add_argument("-b", "--batch-size", default=256, type=int, help="per-process batch")
    p.add_argument("--image-size", default=224, type=int)
    p.add_argument("--lr", "--learning-rate", default=0.1, type=float, help="base lr at batch 256")
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--weight-decay", "--wd", default=1e-4, type=float)
    p.add_argument("--optimizer", default="sgd", choices=["sgd", "adam", "lamb"])
    p.add_argument("--print-freq", "-p", default=10, type=int)
    p.add_argument("--resume", default="", type=str, help="path to a checkpoint")
    p.add_argument("--checkpoint-dir", default=".", type=str)
    p.add_argument("-e", "--evaluate", action="store_true")
    p.add_argument("--pretrained", action="store_true", help="accepted for CLI parity (no downloads)")
    p.add_argument("--opt-level", default="O2")
    p.add_argument("--keep-batchnorm-fp32", default=None)
    p.add_argument("--loss-scale", default=None)
    p.add_argument("--channels-last", default=True, type=lambda s: s.lower() not in ("0", "false", "no"))
    p.add_argument("--sync_bn", action="store_true")
    p.add_argument("--bn", default="fused", choices=["fused", "torch"])
    p.add_argument("--delay-allreduce", action="store_true")
    p.add_argument("--deterministic", action="store_true")
    p.add_argument("--prof", default=-1, type=int, help="stop after this many iterations (profiling)")
    p.add_argument("--seed", default=None, type=int)
    return p.parse_args(argv)


# ----------------------------------------------------------------------------------------------
# data
# ----------------------------------------------------------------------------------------------
class SyntheticSet(torch.utils.data.Dataset):
    """Deterministic uint8 HWC images + labels, the shape a JPEG decode produces."""

    def __init__(self, n, size, seed):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = np.random.default_rng(self.seed * 1000003 + i)
        return g.integers(0, 256, (self.size, self.size, 3), dtype=np.uint8), int(g.integers(0, 1000))


class ImageFolder(torch.utils.data.Dataset):
    """``root/<class>/<image>`` tree decoded with Pillow.  Train: random-resized crop + flip;
    val: resize to size/0.875 + center crop (the reference's torchvision transforms)."""

    EXT = (".jpg", ".jpeg", ".png", ".bmp", ".webp", ".JPEG")

    def __init__(self, root, size, train):
        self.size, self.train = size, train
        classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        self.samples = [(os.path.join(root, c, f), k) for k, c in enumerate(classes)
                        for f in sorted(os.listdir(os.path.join(root, c))) if f.endswith(self.EXT)]

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        from PIL import Image

        path, label = self.samples[i]
        img = Image.open(path).convert("RGB")
        w, h = img.size
        if self.train:
            for _ in range(10):
                area = w * h * random.uniform(0.08, 1.0)
                ar = math.exp(random.uniform(math.log(3 / 4), math.log(4 / 3)))
                cw, ch = int(round(math.sqrt(area * ar))), int(round(math.sqrt(area / ar)))
                if 0 < cw <= w and 0 < ch <= h:
                    x0, y0 = random.randint(0, w - cw), random.randint(0, h - ch)
                    break
            else:
                cw = ch = min(w, h)
                x0, y0 = (w - cw) // 2, (h - ch) // 2
            img = img.resize((self.size, self.size), Image.BILINEAR, box=(x0, y0, x0 + cw, y0 + ch))
            if random.random() < 0.5:
                img = img.transpose(Image.FLIP_LEFT_RIGHT)
        else:
            short = int(self.size / 0.875)
            s = short / min(w, h)
            img = img.resize((max(self.size, round(w * s)), max(self.size, round(h * s))), Image.BILINEAR)
            w, h = img.size
            x0, y0 = (w - self.size) // 2, (h - self.size) // 2
            img = img.crop((x0, y0, x0 + self.size, y0 + self.size))
        return np.asarray(img, dtype=np.uint8), label


def collate(batch):
    """uint8 NHWC batch (normalisation happens on the GPU in the prefetcher)."""
    imgs = torch.from_numpy(np.stack([b[0] for b in batch]))
    return imgs, torch.tensor([b[1] for b in batch], dtype=torch.int64)


def make_loader(ds, batch, workers, shuffle, distributed):
    sampler = torch.utils.data.distributed.DistributedSampler(ds, shuffle=shuffle) if distributed else None
    return torch.utils.data.DataLoader(ds, batch_size=batch, shuffle=(shuffle and sampler is None),
                                       num_workers=workers, pin_memory=torch.cuda.is_available(), sampler=sampler,
                                       collate_fn=collate, drop_last=shuffle, persistent_workers=workers > 0), sampler


class Prefetcher:
    """Upload + normalise batch i+1 on a side stream while batch i trains (reference
    main_amp.py:264-318): NHWC uint8 -> channels_last float normalised, one kernel chain."""

    def __init__(self, loader, device, channels_last):
        self.it = iter(loader)
        self.device = device
        self.cuda = device.type == "cuda"
        self.stream = torch.cuda.Stream() if self.cuda else None
        self.mean = torch.tensor(MEAN, device=device).view(1, 3, 1, 1)
        self.std = torch.tensor(STD, device=device).view(1, 3, 1, 1)
        self.mf = torch.channels_last if channels_last else torch.contiguous_format
        self._load()

    def _prep(self, images, labels):
        x = images.to(self.device, non_blocking=True).permute(0, 3, 1, 2).float()
        x = x.sub_(self.mean).div_(self.std).contiguous(memory_format=self.mf)
        return x, labels.to(self.device, non_blocking=True)

    def _load(self):
        try:
            images, labels = next(self.it)
        except StopIteration:
            self.nxt = (None, None)
            return
        if self.cuda:
            with torch.cuda.stream(self.stream):
                self.nxt = self._prep(images, labels)
        else:
            self.nxt = self._prep(images, labels)

    def next(self):
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.stream)
        x, y = self.nxt
        if x is not None and self.cuda:
            x.record_stream(torch.cuda.current_stream())
            y.record_stream(torch.cuda.current_stream())
        self._load()
        return x, y


# ----------------------------------------------------------------------------------------------
# bookkeeping
# ----------------------------------------------------------------------------------------------
class AverageMeter:
    def __init__(self):
        self.val = self.sum = self.count = 0.0
        self.avg = 0.0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / max(1, self.count)


def accuracy(output, target, topk=(1,)):
    maxk = max(topk)
    _, pred = output.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1))
    return [correct[:k].reshape(-1).float().sum().mul_(100.0 / target.size(0)) for k in topk]


def reduce_mean(t, world):
    if world > 1:
        t = t.clone()
        dist.all_reduce(t)
        t /= world
    return t


def adjust_learning_rate(optimizer, base_lr, epoch, step, len_epoch):
    """Step decay x0.1 at epochs 30 / 60 / 80 with a 5-epoch linear warmup (reference :500-517)."""
    factor = epoch // 30 + (1 if epoch >= 80 else 0)
    lr = base_lr * (0.1 ** factor)
    if epoch < 5:
        lr = lr * float(1 + step + epoch * len_epoch) / (5.0 * len_epoch)
    for g in optimizer.param_groups:
        g["lr"] = lr
    return lr


def save_checkpoint(state, is_best, directory):
    path = os.path.join(directory, "checkpoint.pth.tar")
    torch.save(state, path)
    if is_best:
        shutil.copyfile(path, os.path.join(directory, "model_best.pth.tar"))


# ----------------------------------------------------------------------------------------------
# train / validate
# ----------------------------------------------------------------------------------------------
def train_epoch(loader, model, criterion, optimizer, epoch, args, ctx):
    meters = {k: AverageMeter() for k in ("time", "loss", "top1", "top5")}
    model.train()
    pf = Prefetcher(loader, ctx["device"], args.channels_last)
    x, y = pf.next()
    i = 0
    end = time.time()
    while x is not None:
        if 0 <= args.prof <= i:
            break
        lr = adjust_learning_rate(optimizer, ctx["base_lr"], epoch, i, len(loader))
        out = model(x)
        loss = criterion(out, y)
        optimizer.zero_grad()
        with amp.scale_loss(loss, optimizer) as scaled:
            scaled.backward()
        optimizer.step()
        i += 1
        if i % args.print_freq == 0 or i == len(loader):
            # metrics only at print time: the step itself stays sync-free
            p1, p5 = accuracy(out.float(), y, topk=(1, 5))
            red = reduce_mean(torch.stack([loss.detach().float(), p1, p5]), ctx["world"])
            if ctx["cuda"]:
                torch.cuda.synchronize()
            n = x.size(0)
            meters["loss"].update(red[0].item(), n)
            meters["top1"].update(red[1].item(), n)
            meters["top5"].update(red[2].item(), n)
            meters["time"].update((time.time() - end) / args.print_freq)
            end = time.time()
            if ctx["rank"] == 0:
                print("Epoch: [{0}][{1}/{2}]\tTime {t.val:.3f} ({t.avg:.3f})\tSpeed {3:.1f} ({4:.1f}) img/s\t"
                      "Loss {l.val:.4f} ({l.avg:.4f})\tPrec@1 {p1.val:.3f} ({p1.avg:.3f})\t"
                      "Prec@5 {p5.val:.3f} ({p5.avg:.3f})\tlr {5:.5f}".format(
                          epoch, i, len(loader), ctx["world"] * args.batch_size / max(meters["time"].val, 1e-9),
                          ctx["world"] * args.batch_size / max(meters["time"].avg, 1e-9), lr, t=meters["time"],
                          l=meters["loss"], p1=meters["top1"], p5=meters["top5"]), flush=True)
        x, y = pf.next()
    return meters


@torch.no_grad()
def validate(loader, model, criterion, args, ctx):
    meters = {k: AverageMeter() for k in ("loss", "top1", "top5")}
    model.eval()
    pf = Prefetcher(loader, ctx["device"], args.channels_last)
    x, y = pf.next()
    while x is not None:
        out = model(x)
        loss = criterion(out, y)
        p1, p5 = accuracy(out.float(), y, topk=(1, 5))
        red = reduce_mean(torch.stack([loss.float(), p1, p5]), ctx["world"])
        n = x.size(0)
        meters["loss"].update(red[0].item(), n)
        meters["top1"].update(red[1].item(), n)
        meters["top5"].update(red[2].item(), n)
        x, y = pf.next()
    if ctx["rank"] == 0:
        print(" * Prec@1 {:.3f} Prec@5 {:.3f} Loss {:.4f}".format(meters["top1"].avg, meters["top5"].avg,
                                                                  meters["loss"].avg), flush=True)
    return meters["top1"].avg


def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(local)
    if distributed:
        dist.init_process_group(backend="nccl" if cuda else "gloo", init_method="env://")
    if args.deterministic or args.seed is not None:
        seed = args.seed if args.seed is not None else 0
        torch.manual_seed(seed + rank)
        random.seed(seed + rank)
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
    else:
        torch.backends.cudnn.benchmark = True

    fused_bn = args.bn == "fused" and args.channels_last and cuda
    sync = args.sync_bn and distributed
    # fused NHWC BN: --sync_bn shares the statistics over all ranks inside the fused kernels
    # (bn_group = world); torch BN: apex SyncBatchNorm (detects channels_last memory itself)
    model = getattr(resnet_mod, args.arch)(fused_bn=fused_bn, bn_group=world if (sync and fused_bn) else 1)
    if sync and not fused_bn:
        model = apex.parallel.convert_syncbn_model(model)
    model = model.to(device)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    base_lr = args.lr * args.batch_size * world / 256.0
    if args.optimizer == "sgd":
        optimizer = FusedSGD(model.parameters(), base_lr, momentum=args.momentum, weight_decay=args.weight_decay)
    elif args.optimizer == "adam":
        base_lr *= 0.01
        optimizer = FusedAdam(model.parameters(), lr=base_lr, weight_decay=args.weight_decay)
    else:
        base_lr *= 0.01
        optimizer = FusedLAMB(model.parameters(), lr=base_lr, weight_decay=args.weight_decay)
    model, optimizer = amp.initialize(model, optimizer, opt_level=args.opt_level,
                                      keep_batchnorm_fp32=args.keep_batchnorm_fp32, loss_scale=args.loss_scale,
                                      verbosity=1 if rank == 0 else 0)
    if distributed:
        model = apex.parallel.DistributedDataParallel(model, delay_allreduce=args.delay_allreduce)
    criterion = torch.nn.CrossEntropyLoss().to(device)

    best_prec1 = 0.0
    if args.resume:
        if os.path.isfile(args.resume):
            # our own checkpoint (written by save_checkpoint below): plain tensors and dicts
            ckpt = torch.load(args.resume, map_location=device, weights_only=True)
            args.start_epoch = ckpt["epoch"]
            best_prec1 = ckpt["best_prec1"]
            (model.module if distributed else model).load_state_dict(ckpt["state_dict"])
            optimizer.load_state_dict(ckpt["optimizer"])
            amp.load_state_dict(ckpt["amp"])
            if rank == 0:
                print("=> loaded checkpoint '{}' (epoch {})".format(args.resume, ckpt["epoch"]), flush=True)
        elif rank == 0:
            print("=> no checkpoint found at '{}'".format(args.resume), flush=True)

    if args.data == "synthetic":
        train_set = SyntheticSet(args.iters_per_epoch * args.batch_size * world, args.image_size, 1)
        val_set = SyntheticSet(args.val_iters * args.batch_size * world, args.image_size, 2)
    else:
        train_set = ImageFolder(os.path.join(args.data, "train"), args.image_size, train=True)
        val_set = ImageFolder(os.path.join(args.data, "val"), args.image_size, train=False)
    train_loader, train_sampler = make_loader(train_set, args.batch_size, args.workers, True, distributed)
    val_loader, _ = make_loader(val_set, args.batch_size, args.workers, False, distributed)
    ctx = dict(device=device, cuda=cuda, world=world, rank=rank, base_lr=base_lr)

    if args.evaluate:
        validate(val_loader, model, criterion, args, ctx)
        return best_prec1
    for epoch in range(args.start_epoch, args.epochs):
        if train_sampler is not None:
            train_sampler.set_epoch(epoch)
        train_epoch(train_loader, model, criterion, optimizer, epoch, args, ctx)
        if 0 <= args.prof:
            break
        prec1 = validate(val_loader, model, criterion, args, ctx)
        if rank == 0:
            is_best = prec1 > best_prec1
            best_prec1 = max(prec1, best_prec1)
            save_checkpoint({"epoch": epoch + 1, "arch": args.arch,
                             "state_dict": (model.module if distributed else model).state_dict(),
                             "best_prec1": best_prec1, "optimizer": optimizer.state_dict(),
                             "amp": amp.state_dict()}, is_best, args.checkpoint_dir)
    if distributed:
        dist.destroy_process_group()
    return best_prec1


if __name__ == "__main__":
    main()
