"""Label-smoothed softmax cross-entropy (model: reference apex/contrib/test/xentropy/
test_label_smoothing.py — fused loss vs a torch label-smoothing reference, with padding rows)."""
import pytest
import torch

from apex.contrib.xentropy import SoftmaxCrossEntropyLoss


def _ref_loss(logits, labels, smoothing, padding_idx):
    x = logits.float()
    logp = torch.log_softmax(x, -1)
    nll = -logp.gather(1, labels.view(-1, 1)).squeeze(1)
    smooth = -logp.mean(-1)
    loss = (1 - smoothing) * nll + smoothing * smooth
    return loss.masked_fill(labels == padding_idx, 0.0)


@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_cpu_xentropy(smoothing):
    torch.manual_seed(0)
    logits = torch.randn(12, 37, requires_grad=True)
    labels = torch.randint(0, 37, (12,))
    labels[3] = 0
    loss = SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing, 0, True)
    lr = logits.detach().clone().requires_grad_(True)
    ref = _ref_loss(lr, labels, smoothing, 0)
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)
    g = torch.rand(12)
    loss.backward(g)
    ref.backward(g)
    torch.testing.assert_close(logits.grad, lr.grad, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("classes", [1000, 30528, 50257, 32000])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_gpu_xentropy(classes, dtype, smoothing):
    torch.manual_seed(classes)
    rows = 37
    logits = (torch.randn(rows, classes, device="cuda") * 3).to(dtype).requires_grad_(True)
    labels = torch.randint(1, classes, (rows,), device="cuda")
    labels[::5] = 0  # padding rows
    loss = SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing, 0, True)
    assert loss.dtype == torch.float32
    lr = logits.detach().float().requires_grad_(True)
    ref = _ref_loss(lr, labels, smoothing, 0)
    torch.testing.assert_close(loss, ref, atol=2e-4, rtol=1e-4)
    g = torch.rand(rows, device="cuda")
    loss.backward(g)
    ref.backward(g)
    tol = 1e-6 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(logits.grad.float(), lr.grad, atol=tol, rtol=1e-2)
    assert torch.all(logits.grad[::5] == 0)
