"""gfx950 fp8 conversions inside the multi-tensor engine, the fp8 / model-copy epilogues of the
distributed-optimizer kernels and the in-place Adam undo (reference
apex/contrib/csrc/optimizers/fused_adam_cuda_kernel.cu:390-420 e5m2 convert, :571 reversible
Adam, :657 maybe_adam_undo).  Numerics are pinned to torch's own fp8 casts (bitwise, in range)
and to the fp32 torch math of ``apex.ops.multi_tensor_ref``."""
import pytest
import torch

from apex import amp_C
from apex.ops import multi_tensor_ref as ref

FP8 = [torch.float8_e5m2, torch.float8_e4m3fn]
DEV = "cuda"


def _noop():
    return torch.zeros(1, dtype=torch.int32, device=DEV)


def _in_range(n, dt, seed=0):
    """Values spanning the fp8 normal and subnormal ranges (no overflow)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    fmax = torch.finfo(dt).max
    mant = torch.rand(n, device=DEV, generator=g) * 2 - 1
    expo = torch.randint(-20, 10, (n,), device=DEV, generator=g).float()
    return (mant * torch.pow(2.0, expo)).clamp(-fmax / 2, fmax / 2)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", FP8)
@pytest.mark.parametrize("src", [torch.float32, torch.bfloat16, torch.float16])
def test_cast_to_fp8_matches_torch_gpu(dt, src):
    # sizes cover the 8-wide vector body and the scalar tail; the offset view breaks alignment
    base = _in_range(70001, dt).to(src)
    xs = [base[:4096], base[4096:4096 + 1237], base[5333 + 3:5333 + 3 + 999], base[-7:]]
    outs = [torch.empty(x.shape, dtype=dt, device=DEV) for x in xs]
    amp_C.multi_tensor_cast(65536, _noop(), [xs, outs])
    for x, o in zip(xs, outs):
        assert torch.equal(o.view(torch.uint8), x.to(dt).view(torch.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", FP8)
@pytest.mark.parametrize("dst", [torch.float32, torch.bfloat16])
def test_cast_from_fp8_matches_torch_gpu(dt, dst):
    bits = torch.arange(256, dtype=torch.uint8, device=DEV).repeat(37)
    q = bits.view(dt)
    finite = torch.isfinite(q.float())
    q = q[finite]
    out = torch.empty(q.shape, dtype=dst, device=DEV)
    amp_C.multi_tensor_cast(65536, _noop(), [[q], [out]])
    assert torch.equal(out, q.to(dst))


def _adam_state(n, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    p = torch.randn(n, device=DEV, generator=g)
    m = torch.randn(n, device=DEV, generator=g) * 0.01
    v = torch.rand(n, device=DEV, generator=g) * 1e-4
    gr = torch.randn(n, device=DEV, generator=g).to(torch.bfloat16)
    return gr, p, m, v


@pytest.mark.gpu
@pytest.mark.parametrize("dt", FP8 + [torch.bfloat16])
def test_adam_epilogue_writes_fp8_payload_gpu(dt):
    sizes = [4096, 1000, 64 * 1024 + 5]
    st = [_adam_state(n, i) for i, n in enumerate(sizes)]
    gs, ps, ms, vs = (list(x) for x in zip(*st))
    outs = [torch.empty(n, dtype=dt, device=DEV) for n in sizes]
    rp, rm, rv = [p.clone() for p in ps], [m.clone() for m in ms], [v.clone() for v in vs]
    lr = torch.tensor([1e-3], device=DEV)
    step = torch.tensor([3.0], device=DEV)
    inv = torch.tensor([0.5], device=DEV)
    amp_C.multi_tensor_adam_capturable(65536, _noop(), [gs, ps, ms, vs, outs], lr, 0.9, 0.999, 1e-8, step, 1, 1,
                                       0.01, inv)
    ref.multi_tensor_adam_capturable(65536, _noop(), [gs, rp, rm, rv], lr, 0.9, 0.999, 1e-8, step, 1, 1, 0.01, inv)
    for p, o, r in zip(ps, outs, rp):
        torch.testing.assert_close(p, r, rtol=1e-5, atol=1e-6)
        assert torch.equal(o.view(torch.uint8) if dt in FP8 else o, p.to(dt).view(torch.uint8) if dt in FP8
                           else p.to(dt))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("with_out", [False, True])
def test_adam_undo_restores_pre_step_state_gpu(mode, with_out):
    sizes = [8192, 777, 70000]
    st = [_adam_state(n, 10 + i) for i, n in enumerate(sizes)]
    gs, ps, ms, vs = (list(x) for x in zip(*st))
    before = [(p.clone(), m.clone(), v.clone()) for p, m, v in zip(ps, ms, vs)]
    outs = [torch.empty(n, dtype=torch.bfloat16, device=DEV) for n in sizes]
    lists = [gs, ps, ms, vs] + ([outs] if with_out else [])
    lr = torch.tensor([1e-3], device=DEV)
    step = torch.tensor([5.0], device=DEV)
    inv = torch.tensor([0.25], device=DEV)
    args = (lr, 0.9, 0.999, 1e-8, step, mode, 1, 0.02, inv)
    amp_C.multi_tensor_adam_capturable(65536, _noop(), lists, *args)
    # kernel vs reference math for the undo itself
    cp = [[t.clone() for t in lst] for lst in lists]
    ref.multi_tensor_adam_undo(65536, _noop(), cp, *args)
    amp_C.multi_tensor_adam_undo(65536, _noop(), lists, *args)
    for (p0, m0, v0), p, m, v, rp, rm, rv in zip(before, ps, ms, vs, cp[1], cp[2], cp[3]):
        # kernel vs torch math: fma contraction differs, and (m - (1-b1) g) / b1 cancels
        torch.testing.assert_close(p, rp, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(m, rm, rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(v, rv, rtol=1e-3, atol=3e-8)
        torch.testing.assert_close(p, p0, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(m, m0, rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(v, v0, rtol=1e-3, atol=3e-8)
    if with_out:
        for p, o in zip(ps, outs):
            assert torch.equal(o, p.to(torch.bfloat16))
    # a skipped step (flag set) is not undone
    flag = torch.ones(1, dtype=torch.int32, device=DEV)
    snap = [p.clone() for p in ps]
    amp_C.multi_tensor_adam_undo(65536, flag, lists, *args)
    assert all(torch.equal(a, b) for a, b in zip(ps, snap))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", FP8 + [torch.bfloat16])
def test_lamb_stage2_model_copy_gpu(dt):
    sizes = [1000, 4096, 33]
    ps = [torch.randn(n, device=DEV) for n in sizes]
    us = [torch.randn(n, device=DEV) * 1e-2 for n in sizes]
    outs = [torch.empty(n, dtype=dt, device=DEV) for n in sizes]
    pn = torch.stack([p.norm() for p in ps])
    un = torch.stack([u.norm() for u in us])
    rp = [p.clone() for p in ps]
    amp_C.multi_tensor_lamb_stage2_cuda(65536, _noop(), [ps, us, outs], pn, un, 1e-2, 0.01, False)
    ref.multi_tensor_lamb_stage2_cuda(65536, _noop(), [rp, [u.clone() for u in us]], pn, un, 1e-2, 0.01, False)
    for p, r, o in zip(ps, rp, outs):
        torch.testing.assert_close(p, r, rtol=1e-6, atol=1e-7)
        if dt in FP8:
            assert torch.equal(o.view(torch.uint8), p.to(dt).view(torch.uint8))
        else:
            assert torch.equal(o, p.to(dt))


@pytest.mark.gpu
@pytest.mark.parametrize("beta3", [None, 1.0])
def test_lamb_stage1_beta3_gpu(beta3):
    sizes = [513, 4096]
    gs = [torch.randn(n, device=DEV) for n in sizes]
    ps = [torch.randn(n, device=DEV) for n in sizes]
    ms = [torch.randn(n, device=DEV) * 0.1 for n in sizes]
    vs = [torch.rand(n, device=DEV) * 0.1 for n in sizes]
    us = [torch.empty(n, device=DEV) for n in sizes]
    decay = torch.tensor([0.01, 0.0], device=DEV)
    gn = torch.tensor([0.0], device=DEV)
    cp = [[t.clone() for t in lst] for lst in (gs, ps, ms, vs, us)]
    amp_C.multi_tensor_lamb_stage1_cuda(65536, _noop(), [gs, ps, ms, vs, us], decay, 3, 0.9, 0.99, 1e-6, gn, 1.0,
                                        beta3)
    ref.multi_tensor_lamb_stage1_cuda(65536, _noop(), cp, decay, 3, 0.9, 0.99, 1e-6, gn, 1.0, beta3)
    for a, b in zip(ms + us, cp[2] + cp[4]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
