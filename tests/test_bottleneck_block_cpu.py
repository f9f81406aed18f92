"""CPU tier for the fused bottleneck node plumbing (ops/bottleneck_bn.py): off the GPU the node
is never taken (block_supported is False), and the chained ResNet forward (forward_linked with
BlockLink hand-offs) computes exactly what the plain per-block forward does."""
import torch

from apex.models import resnet50
from apex.models.resnet import Bottleneck
from apex.ops import bottleneck_bn


def test_block_supported_false_on_cpu():
    m = resnet50(fused_bn=True).train()
    x = torch.randn(2, 256, 8, 8).to(memory_format=torch.channels_last)
    blk = m.layer1[1]
    assert isinstance(blk, Bottleneck)
    assert not bottleneck_bn.block_supported(blk, x)
    out, link = blk.forward_linked(x, None)
    if isinstance(out, tuple):  # the per-module path forks a non-final block's output
        out = out[0]
    assert link is None and out.shape == x.shape


def test_chained_forward_matches_sequential_on_cpu():
    torch.manual_seed(0)
    m1 = resnet50(fused_bn=True).train()
    m2 = resnet50(fused_bn=True).train()
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(2, 3, 64, 64)
    y1 = m1(x)  # the fused path's chained block loop (falls back per block on CPU)
    y2 = m2(x)
    torch.testing.assert_close(y1, y2)
    y1.sum().backward()
    assert all(p.grad is not None for p in m1.parameters() if p.requires_grad)


def test_block_link_defaults():
    link = bottleneck_bn.BlockLink()
    assert link.y3 is None and link.bits is None and link.part is None
