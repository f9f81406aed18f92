#!/usr/bin/env python3
"""DCGAN with apex amp and three independently scaled losses (reference examples/dcgan/main_amp.py):
``amp.initialize([netD, netG], [optD, optG], num_losses=3)`` and ``amp.scale_loss(..., loss_id=k)``.
Synthetic 64x64 images (no dataset download); ``--outf`` writes per-epoch checkpoints and the
fixed-noise samples as ``.npy``; ``--netG`` / ``--netD`` resume; runs on the CPU without a GPU."""
import argparse
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from apex import amp  # noqa: E402


def G(nz=100, ngf=64, nc=3):
    return nn.Sequential(
        nn.ConvTranspose2d(nz, ngf * 8, 4, 1, 0, bias=False), nn.BatchNorm2d(ngf * 8), nn.ReLU(True),
        nn.ConvTranspose2d(ngf * 8, ngf * 4, 4, 2, 1, bias=False), nn.BatchNorm2d(ngf * 4), nn.ReLU(True),
        nn.ConvTranspose2d(ngf * 4, ngf * 2, 4, 2, 1, bias=False), nn.BatchNorm2d(ngf * 2), nn.ReLU(True),
        nn.ConvTranspose2d(ngf * 2, ngf, 4, 2, 1, bias=False), nn.BatchNorm2d(ngf), nn.ReLU(True),
        nn.ConvTranspose2d(ngf, nc, 4, 2, 1, bias=False), nn.Tanh())


def D(ndf=64, nc=3):
    return nn.Sequential(
        nn.Conv2d(nc, ndf, 4, 2, 1, bias=False), nn.LeakyReLU(0.2, inplace=True),
        nn.Conv2d(ndf, ndf * 2, 4, 2, 1, bias=False), nn.BatchNorm2d(ndf * 2), nn.LeakyReLU(0.2, inplace=True),
        nn.Conv2d(ndf * 2, ndf * 4, 4, 2, 1, bias=False), nn.BatchNorm2d(ndf * 4), nn.LeakyReLU(0.2, inplace=True),
        nn.Conv2d(ndf * 4, ndf * 8, 4, 2, 1, bias=False), nn.BatchNorm2d(ndf * 8), nn.LeakyReLU(0.2, inplace=True),
        nn.Conv2d(ndf * 8, 1, 4, 1, 0, bias=False))


def weights_init(m):
    """DCGAN init (reference examples/dcgan/main_amp.py weights_init)."""
    name = type(m).__name__
    if "Conv" in name:
        nn.init.normal_(m.weight, 0.0, 0.02)
    elif "BatchNorm" in name:
        nn.init.normal_(m.weight, 1.0, 0.02)
        nn.init.zeros_(m.bias)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", "--batchSize", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20, help="iterations per epoch (synthetic data)")
    ap.add_argument("--niter", type=int, default=1, help="epochs")
    ap.add_argument("--nz", type=int, default=100)
    ap.add_argument("--ngf", type=int, default=64)
    ap.add_argument("--ndf", type=int, default=64)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--beta1", type=float, default=0.5)
    ap.add_argument("--opt-level", "--opt_level", default="O1")
    ap.add_argument("--netG", default="", help="path to a netG checkpoint to resume")
    ap.add_argument("--netD", default="", help="path to a netD checkpoint to resume")
    ap.add_argument("--outf", default="", help="write checkpoints and fake samples (.npy) here")
    ap.add_argument("--manualSeed", type=int, default=None)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args(argv)
    seed = a.manualSeed if a.manualSeed is not None else random.randint(1, 10000)
    random.seed(seed)
    torch.manual_seed(seed)
    dev = torch.device("cuda") if (torch.cuda.is_available() and not a.cpu) else torch.device("cpu")
    netG, netD = G(a.nz, a.ngf).to(dev), D(a.ndf).to(dev)
    netG.apply(weights_init)
    netD.apply(weights_init)
    # our own checkpoints (written below): plain state dicts
    if a.netG:
        netG.load_state_dict(torch.load(a.netG, map_location=dev, weights_only=True))
    if a.netD:
        netD.load_state_dict(torch.load(a.netD, map_location=dev, weights_only=True))
    optD = torch.optim.Adam(netD.parameters(), lr=a.lr, betas=(a.beta1, 0.999))
    optG = torch.optim.Adam(netG.parameters(), lr=a.lr, betas=(a.beta1, 0.999))
    # three losses, each with its own dynamic loss scale (errD_real, errD_fake, errG)
    [netD, netG], [optD, optG] = amp.initialize([netD, netG], [optD, optG], opt_level=a.opt_level, num_losses=3,
                                                verbosity=0)
    crit = nn.BCEWithLogitsLoss()
    g = torch.Generator(device="cpu").manual_seed(seed)
    fixed_noise = torch.randn(a.batch_size, a.nz, 1, 1, generator=g).to(dev)
    for epoch in range(a.niter):
        for i in range(a.iters):
            real = (torch.rand(a.batch_size, 3, 64, 64, generator=g) * 2 - 1).to(dev)
            # (1) D: maximize log(D(x)) + log(1 - D(G(z)))
            netD.zero_grad()
            out = netD(real).view(-1)
            errD_real = crit(out, torch.ones_like(out))
            with amp.scale_loss(errD_real, optD, loss_id=0) as s:
                s.backward()
            D_x = torch.sigmoid(out.float()).mean().item()
            fake = netG(torch.randn(a.batch_size, a.nz, 1, 1, generator=g).to(dev))
            out = netD(fake.detach()).view(-1)
            errD_fake = crit(out, torch.zeros_like(out))
            with amp.scale_loss(errD_fake, optD, loss_id=1) as s:
                s.backward()
            optD.step()
            # (2) G: maximize log(D(G(z)))
            netG.zero_grad()
            out = netD(fake).view(-1)
            errG = crit(out, torch.ones_like(out))
            with amp.scale_loss(errG, optG, loss_id=2) as s:
                s.backward()
            optG.step()
            if i % 5 == 0:
                print("[{}/{}][{}/{}] Loss_D: {:.4f} Loss_G: {:.4f} D(x): {:.4f}".format(
                    epoch, a.niter, i, a.iters, (errD_real + errD_fake).item(), errG.item(), D_x), flush=True)
        if a.outf:
            os.makedirs(a.outf, exist_ok=True)
            with torch.no_grad():
                sample = netG(fixed_noise).float().cpu().numpy()
            np.save(os.path.join(a.outf, "fake_samples_epoch_{:03d}.npy".format(epoch)), sample)
            torch.save(netG.state_dict(), os.path.join(a.outf, "netG_epoch_{}.pth".format(epoch)))
            torch.save(netD.state_dict(), os.path.join(a.outf, "netD_epoch_{}.pth".format(epoch)))
    return errD_real.item() + errD_fake.item(), errG.item()


if __name__ == "__main__":
    main()
