"""Fused bottleneck conv3 backward (csrc/conv/conv3_bwd.hip): bn3's dx as the operand prologue,
conv3's data gradient masked by bn2's ReLU with bn2's backward sums, and conv3's weight
gradient with bn2's apply+ReLU on load — against a float64 PyTorch reference of the same ops."""
import pytest
import torch


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("m", [64 * 40, 64 * 37 + 23, 5000])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gpu_conv3_bwd_fused_matches_float64(m, dtype):
    import apex  # noqa: F401
    from apex import _native

    ext = _native.require("conv").conv
    torch.manual_seed(0)
    dev = "cuda"
    c4, w = 256, 64
    dm = torch.randn(m, c4, device=dev).to(dtype)
    y3 = torch.randn(m, c4, device=dev).to(dtype)
    y2 = torch.randn(m, w, device=dev).to(dtype)
    w3 = (torch.randn(c4, w, device=dev) * 0.1).to(dtype)
    cb3 = torch.randn(3 * c4, device=dev) * 0.5
    c2 = torch.cat([torch.rand(w, device=dev) + 0.5, torch.randn(w, device=dev) * 0.3])
    mean2 = torch.randn(w, device=dev) * 0.1

    dz2, part2, dw3 = ext.conv3_bwd(dm, y3, y2, w3, cb3, c2, mean2)

    A, B, K = (cb3[i * c4:(i + 1) * c4].double() for i in range(3))
    dx3 = (A * dm.double() + B * y3.double() + K).to(dtype).double()
    o2 = y2.double() * c2[:w].double() + c2[w:].double()
    ref_dz2 = torch.where(o2 > 0, dx3 @ w3.double(), torch.zeros_like(o2))
    assert _rel(dz2, ref_dz2) < 8e-3
    g = dz2.double()
    assert _rel(part2[0].sum(0), g.sum(0)) < 1e-4
    assert _rel(part2[1].sum(0), (g * (y2.double() - mean2.double())).sum(0)) < 1e-4
    z2 = torch.relu(o2.float()).to(dtype).double()
    ref_dw3 = dx3.t() @ z2
    assert dw3.shape == (c4, w) and dw3.dtype == dtype
    assert _rel(dw3, ref_dw3) < 8e-3
