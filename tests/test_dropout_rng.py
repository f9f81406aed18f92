"""Graph-safe dropout (apex.ops.dropout_rng): the native dropout kernels read a device step counter
so a hipGraph-captured training step draws fresh masks on every replay, while the forward and the
backward of one step agree and the kernels still match the torch reference of the same hash."""
import pytest
import torch

from apex.ops import dropout_rng


@pytest.fixture
def device_rng():
    dropout_rng.enable(True)
    yield
    dropout_rng.enable(False)


def test_effective_offset_cpu_is_host_offset():
    dropout_rng.enable(True)
    try:
        assert dropout_rng.step_tensor("cpu") is None
        assert dropout_rng.effective_offset(7, "cpu") == 7
    finally:
        dropout_rng.enable(False)
    assert dropout_rng.step_tensor("cpu") is None


@pytest.mark.gpu
def test_gpu_bias_dropout_add_step_counter(device_rng):
    from apex.transformer.functional.fused_bias_dropout_add import fused_bias_dropout_add

    torch.manual_seed(0)
    x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
    r = torch.zeros_like(x)
    y1 = fused_bias_dropout_add(x, None, r, 0.3, True, 11, 5)
    y2 = fused_bias_dropout_add(x, None, r, 0.3, True, 11, 5)
    assert torch.equal(y1, y2), "same step, same (seed, offset): same mask"
    dropout_rng.advance()
    y3 = fused_bias_dropout_add(x, None, r, 0.3, True, 11, 5)
    assert not torch.equal(y1 != 0, y3 != 0), "advanced step must draw a new mask"
    keep = (y3 != 0).float().mean().item()
    assert 0.6 < keep < 0.8
    # the torch reference of the same hash agrees with the kernel at the current step
    from apex import _native

    with _native.reference_mode(True):
        y3r = fused_bias_dropout_add(x, None, r, 0.3, True, 11, 5)
    torch.testing.assert_close(y3.float(), y3r.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.gpu
def test_gpu_graph_replays_draw_fresh_masks_and_backward_agrees(device_rng):
    from apex.transformer.functional.fused_bias_dropout_add import fused_bias_dropout_add

    torch.manual_seed(1)
    x = torch.randn(128, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.zeros(128, 512, device="cuda", dtype=torch.bfloat16)
    g = torch.ones(128, 512, device="cuda", dtype=torch.bfloat16)

    def step():
        dropout_rng.advance()
        y = fused_bias_dropout_add(x, None, r, 0.25, True, 3, 9)
        (dx,) = torch.autograd.grad(y, x, g)
        return y, dx

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        y_s, dx_s = step()
    masks = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        keep_fwd = y_s != 0
        keep_bwd = dx_s != 0
        assert torch.equal(keep_fwd, keep_bwd), "forward and backward of one replay must use one mask"
        masks.append(keep_fwd.clone())
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])


@pytest.mark.gpu
def test_gpu_flash_attention_dropout_uses_step(device_rng):
    from apex import _native
    from apex.ops.attention import flash_attn_func

    torch.manual_seed(2)
    q, k, v = (torch.randn(2, 128, 4, 64, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    o1 = flash_attn_func(q, k, v, dropout_p=0.2, seed=5, offset=1)
    o2 = flash_attn_func(q, k, v, dropout_p=0.2, seed=5, offset=1)
    assert torch.equal(o1, o2)
    dropout_rng.advance()
    o3 = flash_attn_func(q, k, v, dropout_p=0.2, seed=5, offset=1)
    assert not torch.equal(o1, o3)
    go = torch.randn_like(o3)
    dq, dk, dv = torch.autograd.grad(o3, (q, k, v), go)
    qr, kr, vr = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    with _native.reference_mode(True):
        o3r = flash_attn_func(qr, kr, vr, dropout_p=0.2, seed=5, offset=1)
        dqr, dkr, dvr = torch.autograd.grad(o3r, (qr, kr, vr), go)
    for a, b in ((o3, o3r), (dq, dqr), (dk, dkr), (dv, dvr)):
        s = max(1.0, float(b.abs().max()))
        torch.testing.assert_close(a.float() / s, b.float() / s, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
def test_gpu_advance_between_forward_and_backward(device_rng):
    """each forward snapshots the step counter, so an advance() between a forward and
    its backward (gradient accumulation, 1F1B, recompute) cannot change the backward's mask."""
    from apex.ops.attention import flash_attn_func
    from apex.transformer.functional.fused_bias_dropout_add import fused_bias_dropout_add

    torch.manual_seed(4)
    x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.zeros(64, 256, device="cuda", dtype=torch.bfloat16)
    y = fused_bias_dropout_add(x, None, r, 0.3, True, 7, 2)
    dropout_rng.advance()
    (dx,) = torch.autograd.grad(y, x, torch.ones_like(y))
    assert torch.equal(y != 0, dx != 0), "backward must reuse the forward's mask"
    q, k, v = (torch.randn(2, 128, 4, 64, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    go = torch.randn(2, 128, 4, 64, device="cuda", dtype=torch.bfloat16)
    o = flash_attn_func(q, k, v, dropout_p=0.2, seed=5, offset=1)
    ref = torch.autograd.grad(o, (q, k, v), go, retain_graph=True)
    dropout_rng.advance()
    dropout_rng.advance()
    got = torch.autograd.grad(o, (q, k, v), go)
    for a, b in zip(got, ref):
        # (dQ is summed with float atomics: equal up to summation order, far below a mask change)
        torch.testing.assert_close(a.float(), b.float(), atol=2e-3, rtol=1e-2)


@pytest.mark.gpu
def test_gpu_eager_snapshot_not_reused_in_capture(device_rng):
    """a snapshot taken eagerly (warm-up that ends without advance()) must not be
    shared into a graph capture whose body advances only AFTER its dropout calls: every replay
    must still draw a fresh mask."""
    from apex.transformer.functional.fused_bias_dropout_add import fused_bias_dropout_add

    torch.manual_seed(5)
    x = torch.randn(128, 512, device="cuda", dtype=torch.bfloat16)
    r = torch.zeros_like(x)

    def step():
        y = fused_bias_dropout_add(x, None, r, 0.25, True, 3, 9)
        dropout_rng.advance()
        return y

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
        fused_bias_dropout_add(x, None, r, 0.25, True, 3, 9)  # eager snapshot left behind
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        y_s = step()
    masks = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        masks.append((y_s != 0).clone())
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])
