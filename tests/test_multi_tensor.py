"""Multi-tensor op tests (reference tests/L0/run_amp/test_multi_tensor_{scale,axpby,l2norm}.py).

CPU: semantics of the torch reference path (overflow flag, outputs).
GPU: the gfx950 kernels against the fp32 torch reference on ragged tensor lists, all dtype
combinations, vector + scalar tails (odd sizes, misaligned views) and inf/NaN injection."""
import itertools

import pytest
import torch

import apex  # noqa: F401
import amp_C

CHUNK = 2048 * 32
SIZES = [(1, 1), (555, 1), (777, 3), (4096, 2), (65536, 1), (65536 + 3, 2), (333333, 1), (2048 * 32 * 3 + 11, 2)]


def _lists(dev, dtype, sizes, offset=0):
    ts = []
    for n, rep in sizes:
        for _ in range(rep):
            base = torch.randn(n + offset, device=dev, dtype=torch.float32).to(dtype)
            ts.append(base[offset:])
    return ts


def _noop(dev):
    return torch.zeros(1, dtype=torch.int32, device=dev)


# ----------------------------------------------------------------------------- CPU semantics
def test_scale_cpu_overflow_flag():
    a = [torch.ones(10), torch.ones(5)]
    b = [torch.empty(10), torch.empty(5)]
    noop = _noop("cpu")
    amp_C.multi_tensor_scale(CHUNK, noop, [a, b], 0.5)
    assert noop.item() == 0 and torch.allclose(b[0], torch.full((10,), 0.5))
    a[1][2] = float("inf")
    amp_C.multi_tensor_scale(CHUNK, noop, [a, b], 0.5)
    assert noop.item() == 1


def test_l2norm_cpu():
    xs = [torch.randn(100), torch.randn(7)]
    total, per = amp_C.multi_tensor_l2norm(CHUNK, _noop("cpu"), [xs], True)
    ref = torch.cat(xs).norm()
    assert torch.allclose(total, ref.reshape(1), rtol=1e-5)
    assert torch.allclose(per, torch.stack([x.norm() for x in xs]), rtol=1e-5)


def test_axpby_cpu_check_arg():
    x = [torch.randn(8)]
    y = [torch.randn(8)]
    o = [torch.empty(8)]
    noop = _noop("cpu")
    y[0][0] = float("nan")
    amp_C.multi_tensor_axpby(CHUNK, noop, [x, y, o], 2.0, 3.0, 0)  # only x checked
    assert noop.item() == 0
    amp_C.multi_tensor_axpby(CHUNK, noop, [x, y, o], 2.0, 3.0, 1)
    assert noop.item() == 1
    assert torch.allclose(o[0][1:], 2 * x[0][1:] + 3 * y[0][1:])


# ----------------------------------------------------------------------------- GPU numerics
DT = [torch.float32, torch.float16, torch.bfloat16]


def _tol(dt):
    return {torch.float32: 1e-6, torch.float16: 1e-3, torch.bfloat16: 1e-2}[dt]


@pytest.mark.gpu
@pytest.mark.parametrize("din,dout", list(itertools.product(DT, DT)))
@pytest.mark.parametrize("offset", [0, 1])
def test_scale_gpu(din, dout, offset):
    dev = "cuda"
    xs = _lists(dev, din, SIZES, offset)
    ys = [torch.empty_like(x, dtype=dout) for x in xs]
    noop = _noop(dev)
    amp_C.multi_tensor_scale(CHUNK, noop, [xs, ys], 4.0)
    torch.cuda.synchronize()
    assert noop.item() == 0
    for x, y in zip(xs, ys):
        torch.testing.assert_close(y.float(), (x.float() * 4.0).to(dout).float(), rtol=_tol(dout), atol=_tol(dout))
    # overflow injection in the middle of a later chunk of the last tensor
    xs[-1][CHUNK + 5] = float("inf")
    amp_C.multi_tensor_scale(CHUNK, noop, [xs, ys], 4.0)
    torch.cuda.synchronize()
    assert noop.item() == 1
    noop.zero_()
    xs[-1][CHUNK + 5] = float("nan")
    amp_C.multi_tensor_scale(CHUNK, noop, [xs, ys], 4.0)
    assert noop.item() == 1


@pytest.mark.gpu
@pytest.mark.parametrize("dx,dy,do", [(torch.float32,) * 3, (torch.float16, torch.float32, torch.float32),
                                      (torch.bfloat16, torch.float32, torch.bfloat16)])
def test_axpby_gpu(dx, dy, do):
    xs = _lists("cuda", dx, SIZES)
    ys = _lists("cuda", dy, SIZES)
    os_ = [torch.empty_like(x, dtype=do) for x in xs]
    noop = _noop("cuda")
    amp_C.multi_tensor_axpby(CHUNK, noop, [xs, ys, os_], 2.0, -0.5, -1)
    assert noop.item() == 0
    for x, y, o in zip(xs, ys, os_):
        torch.testing.assert_close(o.float(), (2.0 * x.float() - 0.5 * y.float()).to(do).float(),
                                   rtol=_tol(do), atol=_tol(do))
    ys[0][0] = float("inf")
    amp_C.multi_tensor_axpby(CHUNK, noop, [xs, ys, os_], 2.0, -0.5, 0)
    assert noop.item() == 0
    amp_C.multi_tensor_axpby(CHUNK, noop, [xs, ys, os_], 2.0, -0.5, 1)
    assert noop.item() == 1


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("per_tensor", [False, True])
def test_l2norm_gpu(dt, per_tensor):
    xs = _lists("cuda", dt, SIZES)
    noop = _noop("cuda")
    total, per = amp_C.multi_tensor_l2norm(CHUNK, noop, [xs], per_tensor)
    ref_per = torch.stack([x.float().norm() for x in xs])
    torch.testing.assert_close(total, ref_per.norm().reshape(1), rtol=1e-4, atol=1e-4)
    if per_tensor:
        torch.testing.assert_close(per, ref_per, rtol=1e-4, atol=1e-4)
    assert noop.item() == 0
    # deterministic: bitwise equal on repeat
    total2, _ = amp_C.multi_tensor_l2norm(CHUNK, noop, [xs], per_tensor)
    assert torch.equal(total, total2)
    xs[3][0] = float("inf")
    amp_C.multi_tensor_l2norm(CHUNK, noop, [xs], per_tensor)
    assert noop.item() == 1


@pytest.mark.gpu
def test_maxnorm_and_norm_out_gpu():
    xs = _lists("cuda", torch.float32, SIZES)
    noop = _noop("cuda")
    total, per = amp_C.multi_tensor_maxnorm(CHUNK, noop, [xs], True)
    ref = torch.stack([x.abs().max() for x in xs])
    torch.testing.assert_close(per, ref)
    torch.testing.assert_close(total, ref.max().reshape(1))
    out = torch.rand(len(xs), device="cuda")
    old = out.clone()
    amp_C.multi_tensor_norm_out(CHUNK, noop, [xs], out, 0.9, 0.1, 2)
    exp = torch.sqrt(0.9 * old * old + 0.1 * torch.stack([(x * x).sum() for x in xs]))
    torch.testing.assert_close(out, exp, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_l2norm_scale_gpu():
    xs = _lists("cuda", torch.float16, SIZES)
    ys = [torch.empty_like(x, dtype=torch.float32) for x in xs]
    noop = _noop("cuda")
    total, _ = amp_C.multi_tensor_l2norm_scale(CHUNK, noop, [xs, ys], 0.25, False)
    torch.testing.assert_close(total, torch.stack([x.float().norm() for x in xs]).norm().reshape(1), rtol=1e-4,
                               atol=1e-4)
    for x, y in zip(xs, ys):
        torch.testing.assert_close(y, x.float() * 0.25)


@pytest.mark.gpu
def test_check_finite_and_cache_gpu():
    xs = _lists("cuda", torch.bfloat16, SIZES)
    noop = _noop("cuda")
    amp_C.multi_tensor_check_finite(CHUNK, noop, [xs])
    n1 = amp_C.mta_cache_size()
    amp_C.multi_tensor_check_finite(CHUNK, noop, [xs])
    # same list -> cached work table reused (an earlier test may already own this key, when the
    # caching allocator hands back identical addresses, so only the second call is checked)
    assert amp_C.mta_cache_size() == n1
    assert noop.item() == 0
    xs[-1][-1] = float("-inf")
    amp_C.multi_tensor_check_finite(CHUNK, noop, [xs])
    assert noop.item() == 1


@pytest.mark.gpu
def test_update_scale_device():
    from apex.ops import multi_tensor_ref as ref

    for dynamic in (True, False):
        for ovf in (0, 1):
            st_g = torch.tensor([65536.0, 1.0, 1999.0, 0.0], device="cuda")
            st_c = st_g.cpu().clone()
            o_g = torch.tensor([ovf], dtype=torch.int32, device="cuda")
            s_g = torch.zeros(1, dtype=torch.int32, device="cuda")
            s_c = torch.zeros(1, dtype=torch.int32)
            amp_C.amp_update_scale_(o_g, s_g, st_g, 2.0, 0.5, 2000, 0.0, 2.0 ** 24, dynamic)
            ref.amp_update_scale_(o_g.cpu(), s_c, st_c, 2.0, 0.5, 2000, 0.0, 2.0 ** 24, dynamic)
            torch.testing.assert_close(st_g.cpu(), st_c)
            assert s_g.item() == s_c.item()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_l2norm_mp_inf_in_early_chunk_many_chunks(device):
    """multi_tensor_l2norm_mp (skip-on-noop reduction) with far more chunks than blocks and an inf
    in the first chunk: blocks that start after the flag is raised skip their chunks, the
    launch still terminates promptly, reports the skipped result (norm 0, flag set), and the
    next clean launch over the same table gets the exact norm (fresh partial tags)."""
    import time

    chunk = 64  # tiny chunks: ~16k chunks, many per block
    xs = [torch.randn(1 << 20, device=device), torch.randn(3000, device=device)]
    ref = torch.cat([x.reshape(-1) for x in xs]).norm()
    noop = _noop(device)
    total, _ = amp_C.multi_tensor_l2norm_mp(chunk, noop, [xs], False)
    torch.testing.assert_close(total, ref.reshape(1), rtol=1e-4, atol=1e-4)
    for rep in range(3):
        xs[0][1] = float("inf")
        noop.zero_()
        t0 = time.time()
        total, per = amp_C.multi_tensor_l2norm_mp(chunk, noop, [xs], True)
        if device == "cuda":
            torch.cuda.synchronize()
        assert time.time() - t0 < 5.0, "finalizer waited on partials nobody wrote"
        assert int(noop.item()) == 1
        assert float(total) == 0.0 and torch.count_nonzero(per) == 0
        xs[0][1] = 0.5
        noop.zero_()
        total, per = amp_C.multi_tensor_l2norm_mp(chunk, noop, [xs], True)
        exp = torch.cat([x.reshape(-1) for x in xs]).norm()
        torch.testing.assert_close(total, exp.reshape(1), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(per, torch.stack([x.norm() for x in xs]), rtol=1e-4, atol=1e-4)
        assert int(noop.item()) == 0


@pytest.mark.gpu
def test_new_addresses_patch_the_cached_table_gpu():
    """Gradients set to None between steps come back at new addresses: a structurally identical
    list patches the cached table's address rows (mta_host.cpp) instead of adding a table, and the
    op reads the NEW tensors (not the old addresses)."""
    amp_C.mta_cache_clear()
    noop = _noop("cuda")
    keep = []
    for step in range(4):
        xs = _lists("cuda", torch.float32, SIZES)
        keep.append(xs)  # hold the old lists so the allocator cannot hand the same addresses back
        ys = [torch.empty_like(x) for x in xs]
        amp_C.multi_tensor_scale(CHUNK, noop, [xs, ys], 2.0)
        for x, y in zip(xs, ys):
            torch.testing.assert_close(y, x * 2.0)
        if step == 0:
            n1 = amp_C.mta_cache_size()
    assert amp_C.mta_cache_size() == n1
    # an exact repeat of an older list is still correct (it patches back)
    ys = [torch.empty_like(x) for x in keep[0]]
    amp_C.multi_tensor_scale(CHUNK, noop, [keep[0], ys], 3.0)
    for x, y in zip(keep[0], ys):
        torch.testing.assert_close(y, x * 3.0)
    assert noop.item() == 0


@pytest.mark.gpu
def test_table_hit_during_capture_is_pinned_gpu():
    """A table first built EAGERLY on the capture stream (warm-up) and then hit while a graph is
    captured must be pinned: a later eager call with the same structure but new tensors may not
    patch its address rows, or the next replay would read the new tensors (mta_host.cpp)."""
    amp_C.mta_cache_clear()
    s = torch.cuda.Stream()
    noop = _noop("cuda")
    xs = _lists("cuda", torch.float32, SIZES)
    ys = [torch.empty_like(x) for x in xs]
    with torch.cuda.stream(s):
        amp_C.multi_tensor_scale(CHUNK, noop, [xs, ys], 2.0)  # eager warm-up builds the table
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        amp_C.multi_tensor_scale(CHUNK, noop, [xs, ys], 2.0)  # cache hit while capturing
    # eager call on the same stream, same structure, new tensors
    xs2 = _lists("cuda", torch.float32, SIZES)
    ys2 = [torch.empty_like(x) for x in xs2]
    with torch.cuda.stream(s):
        amp_C.multi_tensor_scale(CHUNK, noop, [xs2, ys2], 2.0)
    s.synchronize()
    for x, y in zip(xs2, ys2):
        torch.testing.assert_close(y, x * 2.0)
    for x in xs:
        x.mul_(-1.0)
    for y in ys:
        y.zero_()
    g.replay()
    torch.cuda.synchronize()
    for x, y in zip(xs, ys):
        torch.testing.assert_close(y, x * 2.0)
    assert noop.item() == 0
