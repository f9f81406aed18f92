"""Bottleneck / SpatialBottleneck.  Model: reference apex/contrib/bottleneck/test.py and
bottleneck_module_test.py (fused block vs the plain module path; spatial split over ranks vs
the whole image on one rank, outputs and gradients)."""
import copy

import pytest
import torch

from apex.contrib.bottleneck import Bottleneck, SpatialBottleneck
from tests._dist_utils import run_multiprocess


def _randomize_bn(block):
    g = torch.Generator().manual_seed(1)
    for bn in (block.bn1, block.bn2, block.bn3) + ((block.downsample[1],) if block.downsample is not None else ()):
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.2, 0.2, generator=g)
        bn.running_mean.uniform_(-0.2, 0.2, generator=g)
        bn.running_var.uniform_(0.5, 1.5, generator=g)


@pytest.mark.parametrize("stride,cin", [(1, 64), (2, 32)])
def test_fused_matches_modules(stride, cin):
    torch.manual_seed(0)
    blk = Bottleneck(cin, 16, 64, stride=stride)
    _randomize_bn(blk)
    fused = copy.deepcopy(blk)
    fused.use_cudnn = True
    x = torch.randn(2, cin, 12, 12, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    y = blk(x)
    y2 = fused(x2)
    torch.testing.assert_close(y, y2, atol=1e-5, rtol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, atol=1e-5, rtol=1e-4)
    for a, b in zip(blk.w_conv, fused.w_conv):
        torch.testing.assert_close(a.grad, b.grad, atol=1e-4, rtol=1e-4)


def test_explicit_nhwc():
    torch.manual_seed(0)
    ref = Bottleneck(32, 16, 64, stride=2)
    _randomize_bn(ref)
    nhwc = Bottleneck(32, 16, 64, stride=2, use_cudnn=True, explicit_nhwc=True)
    nhwc.load_state_dict({k: (v.permute(0, 2, 3, 1) if v.dim() == 4 else v) for k, v in ref.state_dict().items()})
    x = torch.randn(2, 32, 8, 8)
    y = ref(x)
    y2 = nhwc(x.permute(0, 2, 3, 1).contiguous())
    torch.testing.assert_close(y2, y.permute(0, 2, 3, 1), atol=1e-5, rtol=1e-4)


def _spatial_worker(rank, world, use_cudnn):
    torch.manual_seed(0)
    full = Bottleneck(32, 16, 32)
    _randomize_bn(full)
    sp = SpatialBottleneck(32, 16, 32, use_cudnn=use_cudnn, spatial_group_size=world)
    sp.load_state_dict(full.state_dict())
    x = torch.randn(2, 32, 8, 6, requires_grad=True)
    y = full(x)
    g = torch.randn_like(y)
    y.backward(g)
    h = 8 // world
    xs = x.detach()[:, :, rank * h:(rank + 1) * h].clone().requires_grad_(True)
    ys = sp(xs)
    torch.testing.assert_close(ys, y[:, :, rank * h:(rank + 1) * h], atol=1e-5, rtol=1e-4)
    ys.backward(g[:, :, rank * h:(rank + 1) * h])
    torch.testing.assert_close(xs.grad, x.grad[:, :, rank * h:(rank + 1) * h], atol=1e-5, rtol=1e-4)
    # weight grads are per-rank partial sums: all-reduce and compare
    for a, b in zip(sp.w_conv, full.w_conv):
        ga = a.grad.clone()
        torch.distributed.all_reduce(ga)
        torch.testing.assert_close(ga, b.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("use_cudnn", [False, True])
def test_spatial_bottleneck_two_ranks(use_cudnn):
    run_multiprocess(_spatial_worker, world=2, args=(use_cudnn,))
