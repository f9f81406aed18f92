#!/usr/bin/env python3
"""DCGAN with apex amp and three independently scaled losses (reference examples/dcgan/main_amp.py):
``amp.initialize([netD, netG], [optD, optG], num_losses=3)`` and ``amp.scale_loss(..., loss_id=k)``.
Synthetic 64x64 images (no dataset download)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--opt-level", default="O1")
    a = ap.parse_args()
    dev = torch.device("cuda")
    netG, netD = G().to(dev), D().to(dev)
    optD = torch.optim.Adam(netD.parameters(), lr=2e-4, betas=(0.5, 0.999))
    optG = torch.optim.Adam(netG.parameters(), lr=2e-4, betas=(0.5, 0.999))
    [netD, netG], [optD, optG] = amp.initialize([netD, netG], [optD, optG], opt_level=a.opt_level, num_losses=3)
    crit = nn.BCEWithLogitsLoss()
    real = torch.rand(a.batch_size, 3, 64, 64, device=dev) * 2 - 1
    for i in range(a.iters):
        netD.zero_grad()
        out = netD(real).view(-1)
        errD_real = crit(out, torch.ones_like(out))
        with amp.scale_loss(errD_real, optD, loss_id=0) as s:
            s.backward()
        fake = netG(torch.randn(a.batch_size, 100, 1, 1, device=dev))
        out = netD(fake.detach()).view(-1)
        errD_fake = crit(out, torch.zeros_like(out))
        with amp.scale_loss(errD_fake, optD, loss_id=1) as s:
            s.backward()
        optD.step()
        netG.zero_grad()
        out = netD(fake).view(-1)
        errG = crit(out, torch.ones_like(out))
        with amp.scale_loss(errG, optG, loss_id=2) as s:
            s.backward()
        optG.step()
        if i % 5 == 0:
            print("[{}/{}] Loss_D: {:.4f} Loss_G: {:.4f}".format(i, a.iters, (errD_real + errD_fake).item(),
                                                                errG.item()), flush=True)


if __name__ == "__main__":
    main()
