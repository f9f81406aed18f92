"""CPU tier for the fused bottleneck node plumbing (ops/bottleneck_bn.py): off the GPU the node
is never taken (block_supported is False); the fused-BN model matches the plain torch ResNet."""
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


def test_fused_model_matches_plain_resnet_on_cpu():
    """Two different code paths: the fused-BN model (linked block walk, fused NHWC batch-norm
    modules falling back to their torch reference math on the CPU) against the plain
    torchvision-layout ResNet-50 (nn.BatchNorm2d + ReLU) with the same state dict — output,
    every parameter gradient and the running statistics."""
    torch.manual_seed(0)
    # float64 models: a random-init ResNet-50 at batch 2 amplifies fp32 summation-order noise in
    # its BN backward to ~1-3 % per gradient, which would hide a real difference; the fused
    # modules' CPU math agrees with the plain model to ~1e-6 in float64 (fp32 internals)
    plain = resnet50().train().double()
    fused = resnet50(fused_bn=True).train().double()
    fused.load_state_dict(plain.state_dict())
    x = torch.randn(2, 3, 64, 64, dtype=torch.float64)
    tgt = torch.randint(0, 1000, (2,))
    y1, y2 = fused(x), plain(x)
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))  # noqa: E731
    assert rel(y1, y2) < 1e-4, rel(y1, y2)
    torch.nn.functional.cross_entropy(y1, tgt).backward()
    torch.nn.functional.cross_entropy(y2, tgt).backward()
    g2 = dict(plain.named_parameters())
    for n, p in fused.named_parameters():
        assert rel(p.grad, g2[n].grad) < 1e-4, (n, rel(p.grad, g2[n].grad))
    b2 = dict(plain.named_buffers())
    for n, b in fused.named_buffers():
        if b.dtype.is_floating_point:
            torch.testing.assert_close(b, b2[n], atol=1e-5, rtol=1e-4, msg=n)


def test_module_hooks_run_the_layers_unlinked_on_cpu():
    """a forward hook on a block makes the model call the layers through __call__
    (the hook fires; the linked walk would bypass it) with unchanged results."""
    torch.manual_seed(1)
    m = resnet50(fused_bn=True).train()
    x = torch.randn(2, 3, 64, 64)
    y0 = m(x)
    seen = []
    h = m.layer2[1].register_forward_hook(lambda mod, inp, out: seen.append(1))
    try:
        y1 = m(x)
    finally:
        h.remove()
    assert seen == [1]
    torch.testing.assert_close(y0, y1)


def test_block_link_defaults():
    link = bottleneck_bn.BlockLink()
    assert link.y3 is None and link.bits is None and link.part is None
