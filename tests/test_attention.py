"""Fused attention: flash kernels, multihead_attn modules, FMHA.

Model: reference apex/contrib/test/multihead_attn/test_self_multihead_attn.py (fast impl vs
default impl, outputs and input grads), test_encdec_multihead_attn.py, test_mha_fused_softmax.py,
and apex/contrib/test/fmha/test_fmha.py (packed varlen qkv vs per-sequence python attention).
GPU tiers compare the gfx950 kernels against fp32 torch math of the same op, including the
dropout mask (the kernels' counter-based hash is mirrored in python)."""
import math

import pytest
import torch
import torch.nn.functional as F

from apex.ops.attention import dropout_keep_mask, flash_attn_func


def naive(q, k, v, scale, causal=False, bias=None, keep=None, p=0.0):
    # q [b, sq, h, d]; k, v [b, sk, hk, d]
    rep = q.size(2) // k.size(2)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    s = qf @ kf.transpose(-1, -2) * scale
    if bias is not None:
        s = s + bias
    if causal:
        s = s.masked_fill(torch.ones(s.shape[-2:], dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    pr = torch.softmax(s, -1)
    if keep is not None:
        # the kernels' exact keep rate (16-bit threshold): 65536 / (65536 - floor(p * 65536))
        pr = pr * keep * (65536.0 / (65536 - int(p * 65536.0)))
    return (pr @ vf).transpose(1, 2)


@pytest.mark.parametrize("causal", [False, True])
def test_cpu_reference_matches_naive(causal):
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 9, 4, 16, requires_grad=True) for _ in range(3))
    bias = torch.randn(2, 1, 1, 9)
    out = flash_attn_func(q, k, v, causal=causal, bias=bias)
    ref = naive(q, k, v, 0.25, causal, bias)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(out)
    gq = torch.autograd.grad(out, (q, k, v), g)
    gr = torch.autograd.grad(ref, (q, k, v), g)
    for a, b in zip(gq, gr):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


def test_cpu_gqa_varlen_dropout_semantics():
    torch.manual_seed(1)
    lens = [5, 11, 3]
    cu = torch.tensor([0, 5, 16, 19], dtype=torch.int32)
    q = torch.randn(19, 4, 16)
    k = torch.randn(19, 2, 16)
    v = torch.randn(19, 2, 16)
    out = flash_attn_func(q, k, v, cu_seqlens_q=cu, cu_seqlens_k=cu, dropout_p=0.3, seed=7, offset=3)
    for bi, (a, b) in enumerate(zip(cu[:-1].tolist(), cu[1:].tolist())):
        bh = bi * 4 + torch.arange(4)
        keep = dropout_keep_mask(7, 3, bh, lens[bi], lens[bi], 0.3).view(1, 4, lens[bi], lens[bi])
        ref = naive(q[a:b][None], k[a:b][None], v[a:b][None], 0.25, keep=keep.float(), p=0.3)[0]
        torch.testing.assert_close(out[a:b], ref, atol=1e-5, rtol=1e-5)
    frac = dropout_keep_mask(1, 2, torch.arange(8), 64, 64, 0.25).float().mean().item()
    assert abs(frac - 0.75) < 0.02


def _mha_pair(cls, **kw):
    from apex.contrib.multihead_attn import EncdecMultiheadAttn, SelfMultiheadAttn  # noqa: F401

    torch.manual_seed(2)
    fast = cls(64, 4, impl="fast", **kw)
    default = cls(64, 4, impl="default", **kw)
    default.load_state_dict(fast.state_dict(), strict=False)
    return fast, default


@pytest.mark.parametrize("bias,norm_add,mask", [(False, False, None), (True, False, "pad"), (True, True, "time"),
                                                (False, True, "pad")])
def test_cpu_self_mha_fast_vs_default(bias, norm_add, mask):
    from apex.contrib.multihead_attn import SelfMultiheadAttn

    fast = SelfMultiheadAttn(64, 4, bias=bias, include_norm_add=norm_add, impl="fast")
    default = SelfMultiheadAttn(64, 4, bias=bias, include_norm_add=norm_add, impl="default")
    sd = fast.state_dict()
    if norm_add:
        sd = {k: v for k, v in sd.items() if not k.startswith("lyr_nrm")}
    default.load_state_dict(sd, strict=False)
    x = torch.randn(10, 3, 64, requires_grad=True)
    kpm = tm = None
    if mask == "pad":
        kpm = torch.zeros(3, 10, dtype=torch.bool)
        kpm[1, 7:] = True
    elif mask == "time":
        tm = torch.ones(10, 10, dtype=torch.bool).triu(1)
    y1, _ = fast(x, x, x, key_padding_mask=kpm, attn_mask=tm, is_training=False)
    y2, _ = default(x, x, x, key_padding_mask=kpm, attn_mask=tm, is_training=False)
    torch.testing.assert_close(y1, y2, atol=1e-5, rtol=1e-4)
    g1 = torch.autograd.grad(y1.sum(), x)[0]
    g2 = torch.autograd.grad(y2.sum(), x)[0]
    torch.testing.assert_close(g1, g2, atol=1e-5, rtol=1e-4)


def test_cpu_encdec_mha_and_softmax_dropout():
    from apex.contrib.multihead_attn import EncdecMultiheadAttn, fast_mask_softmax_dropout_func

    fast = EncdecMultiheadAttn(64, 8, impl="fast")
    default = EncdecMultiheadAttn(64, 8, impl="default")
    default.load_state_dict(fast.state_dict())
    q = torch.randn(6, 2, 64)
    kv = torch.randn(9, 2, 64)
    kpm = torch.zeros(2, 9, dtype=torch.bool)
    kpm[0, 5:] = True
    y1, _ = fast(q, kv, kv, key_padding_mask=kpm, is_training=False)
    y2, _ = default(q, kv, kv, key_padding_mask=kpm, is_training=False)
    torch.testing.assert_close(y1, y2, atol=1e-5, rtol=1e-4)
    s = torch.randn(2 * 8, 6, 9, requires_grad=True)
    out = fast_mask_softmax_dropout_func(False, 8, s, kpm, False, 0.0)
    ref = torch.softmax(s.view(2, 8, 6, 9).masked_fill(kpm.view(2, 1, 1, 9), float("-inf")), -1).view(16, 6, 9)
    torch.testing.assert_close(out, ref)
    gs = torch.autograd.grad(out.sum() + (out * out).sum(), s)[0]
    gr = torch.autograd.grad(ref.sum() + (ref * ref).sum(), s)[0]
    torch.testing.assert_close(gs, gr, atol=1e-6, rtol=1e-5)


def test_cpu_fmha_module():
    from apex.contrib.fmha import FMHA

    class Cfg:
        attention_probs_dropout_prob = 0.0
        num_attention_heads = 2
        hidden_size = 64

    cu = torch.tensor([0, 4, 10], dtype=torch.int32)
    qkv = torch.randn(10, 3 * 64, requires_grad=True)
    out = FMHA(Cfg())(qkv, cu, 6, is_training=False)
    x = qkv.view(10, 3, 2, 32)
    for a, b in ((0, 4), (4, 10)):
        ref = naive(x[a:b, 0][None], x[a:b, 1][None], x[a:b, 2][None], 32 ** -0.5)[0].reshape(b - a, 64)
        torch.testing.assert_close(out[a:b], ref, atol=1e-5, rtol=1e-5)
    out.sum().backward()
    assert qkv.grad is not None and torch.isfinite(qkv.grad).all()


# ------------------------------------------------------------------------------------------
# GPU: gfx950 kernels vs fp32 math
# ------------------------------------------------------------------------------------------
def _close(got, ref, tol):
    s = max(1.0, float(ref.abs().max()))
    torch.testing.assert_close(got.float() / s, ref.float() / s, atol=tol, rtol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
def test_gpu_flash_fwd_bwd(d, dtype, causal):
    import apex

    assert apex._native.submodule("attn") is not None, "attention kernels not built"
    torch.manual_seed(d)
    b, sq, sk, h = 2, 200, 200 if causal else 333, 4
    q = torch.randn(b, sq, h, d, device="cuda", dtype=dtype, requires_grad=True)
    k = torch.randn(b, sk, h, d, device="cuda", dtype=dtype, requires_grad=True)
    v = torch.randn(b, sk, h, d, device="cuda", dtype=dtype, requires_grad=True)
    scale = d ** -0.5
    out = flash_attn_func(q, k, v, causal=causal)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = naive(qr, kr, vr, scale, causal)
    tol = 2e-2
    _close(out, ref, tol)
    g = torch.randn_like(ref)
    out.backward(g.to(dtype))
    ref.backward(g)
    _close(q.grad, qr.grad, tol)
    _close(k.grad, kr.grad, tol)
    _close(v.grad, vr.grad, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("qs", ["32", "64"])
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("causal,sq,sk", [(False, 200, 333), (True, 200, 200), (False, 40, 97), (True, 40, 40)])
def test_gpu_flash_bwd_dkdv_slices(qs, d, causal, sq, sk, monkeypatch):
    """dK/dV kernel with 32- and 64-query LDS slices forced (default: 64 at head dim 128, 32
    below): ragged query counts end a 64-slice after its first 32-query half."""
    monkeypatch.setenv("APEX_ATTN_DKDV_QS", qs)
    torch.manual_seed(d + sq)
    b, h, dtype = 2, 3, torch.bfloat16
    q = torch.randn(b, sq, h, d, device="cuda", dtype=dtype, requires_grad=True)
    k = torch.randn(b, sk, h, d, device="cuda", dtype=dtype, requires_grad=True)
    v = torch.randn(b, sk, h, d, device="cuda", dtype=dtype, requires_grad=True)
    out = flash_attn_func(q, k, v, causal=causal)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = naive(qr, kr, vr, d ** -0.5, causal)
    g = torch.randn_like(ref)
    out.backward(g.to(dtype))
    ref.backward(g)
    for a, r in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        _close(a, r, 2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("d,causal,sq,sk", [(64, True, 200, 200), (128, False, 150, 333), (64, False, 70, 45)])
def test_gpu_flash_dropout_causal_ragged(d, causal, sq, sk):
    """Dropout (counter-hash decisions, regenerated in the backward) with causal masking and
    ragged key blocks, against the fp32 reference with the same keep mask."""
    torch.manual_seed(d + sq)
    b, h, dtype, p = 2, 3, torch.bfloat16, 0.25
    q = torch.randn(b, sq, h, d, device="cuda", dtype=dtype, requires_grad=True)
    k = torch.randn(b, sk, h, d, device="cuda", dtype=dtype, requires_grad=True)
    v = torch.randn(b, sk, h, d, device="cuda", dtype=dtype, requires_grad=True)
    out = flash_attn_func(q, k, v, dropout_p=p, causal=causal, seed=21, offset=3)
    keep = dropout_keep_mask(21, 3, torch.arange(b * h), sq, sk, p, "cuda").view(b, h, sq, sk).float()
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = naive(qr, kr, vr, d ** -0.5, causal, keep=keep, p=p)
    _close(out, ref, 2e-2)
    g = torch.randn_like(ref)
    out.backward(g.to(dtype))
    ref.backward(g)
    for a, r in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        _close(a, r, 3e-2)


@pytest.mark.gpu
def test_gpu_flash_bias_gqa_dropout_varlen():
    torch.manual_seed(5)
    dtype = torch.bfloat16
    # bias + GQA + dropout, padded layout
    b, s, h, hk, d = 2, 150, 8, 2, 64
    q = torch.randn(b, s, h, d, device="cuda", dtype=dtype, requires_grad=True)
    k = torch.randn(b, s, hk, d, device="cuda", dtype=dtype, requires_grad=True)
    v = torch.randn(b, s, hk, d, device="cuda", dtype=dtype, requires_grad=True)
    bias = torch.zeros(b, 1, 1, s, device="cuda")
    bias[1, :, :, 100:] = float("-inf")
    bias[0] += torch.randn(1, 1, s, device="cuda")
    p = 0.2
    out = flash_attn_func(q, k, v, dropout_p=p, bias=bias, seed=11, offset=5)
    bh = torch.arange(b * h)
    keep = dropout_keep_mask(11, 5, bh, s, s, p, "cuda").view(b, h, s, s).float()
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = naive(qr, kr, vr, d ** -0.5, bias=bias, keep=keep, p=p)
    _close(out, ref, 2e-2)
    g = torch.randn_like(ref)
    out.backward(g.to(dtype))
    ref.backward(g)
    for a, r in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        _close(a, r, 3e-2)
    # varlen packed
    lens = [17, 130, 64, 1]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    tot = sum(lens)
    q = torch.randn(tot, 4, 128, device="cuda", dtype=dtype, requires_grad=True)
    k = torch.randn(tot, 4, 128, device="cuda", dtype=dtype, requires_grad=True)
    v = torch.randn(tot, 4, 128, device="cuda", dtype=dtype, requires_grad=True)
    out = flash_attn_func(q, k, v, cu_seqlens_q=cu, cu_seqlens_k=cu, causal=True)
    g = torch.randn_like(out)
    out.backward(g)
    c = cu.tolist()
    for i in range(len(lens)):
        a, e = c[i], c[i + 1]
        qr, kr, vr = (t.detach()[a:e].float()[None].requires_grad_(True) for t in (q, k, v))
        ref = naive(qr, kr, vr, 128 ** -0.5, causal=True)
        _close(out[a:e][None], ref, 2e-2)
        ref.backward(g[a:e][None].float())
        _close(q.grad[a:e][None], qr.grad, 3e-2)
        _close(k.grad[a:e][None], kr.grad, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("norm_add", [False, True])
def test_gpu_self_mha_fast_vs_default(norm_add):
    from apex.contrib.multihead_attn import SelfMultiheadAttn

    torch.manual_seed(3)
    fast = SelfMultiheadAttn(1024, 16, bias=True, include_norm_add=norm_add, impl="fast").cuda().half()
    default = SelfMultiheadAttn(1024, 16, bias=True, include_norm_add=norm_add, impl="default").cuda().half()
    sd = {k: v for k, v in fast.state_dict().items() if not k.startswith("lyr_nrm")}
    default.load_state_dict(sd, strict=False)
    x = torch.randn(128, 8, 1024, device="cuda", dtype=torch.half, requires_grad=True)
    kpm = torch.zeros(8, 128, dtype=torch.bool, device="cuda")
    kpm[3, 90:] = True
    y1, _ = fast(x, x, x, key_padding_mask=kpm, is_training=False)
    y2, _ = default(x, x, x, key_padding_mask=kpm, is_training=False)
    _close(y1, y2, 2e-2)
    g = torch.randn_like(y1)
    g1 = torch.autograd.grad(y1, x, g)[0]
    g2 = torch.autograd.grad(y2, x, g)[0]
    _close(g1, g2, 3e-2)


@pytest.mark.gpu
def test_gpu_fmha_vs_reference():
    from apex.contrib.fmha import FMHA

    class Cfg:
        attention_probs_dropout_prob = 0.0
        num_attention_heads = 16
        hidden_size = 1024

    torch.manual_seed(4)
    lens = [128, 384, 77, 512]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    qkv = torch.randn(sum(lens), 3 * 1024, device="cuda", dtype=torch.half, requires_grad=True)
    out = FMHA(Cfg())(qkv, cu, 512, is_training=True)
    g = torch.randn_like(out)
    out.backward(g)
    x = qkv.detach().view(-1, 3, 16, 64)
    c = cu.tolist()
    for i in range(len(lens)):
        a, e = c[i], c[i + 1]
        xr = x[a:e].float().requires_grad_(True)
        ref = naive(xr[:, 0][None], xr[:, 1][None], xr[:, 2][None], 0.125)[0].reshape(e - a, 1024)
        _close(out[a:e], ref, 2e-2)
        ref.backward(g[a:e].float())
        _close(qkv.grad[a:e].view(-1, 3, 16, 64), xr.grad, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_gpu_packed_qkv_self_attention_matches_views(causal):
    """Megatron [s, b, h, 3d] packed path (strided q/k/v, in-place [s, b] context, one d(QKV)
    buffer) against flash_attn_func on the same views."""
    from apex.ops.attention import packed_qkv_self_attention

    torch.manual_seed(7)
    s, b, h, d = 200, 3, 4, 64
    mixed = torch.randn(s, b, h, 3 * d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    bias = None
    if not causal:
        bias = torch.zeros(b, 1, 1, s, device="cuda")
        bias[1, ..., 150:] = -10000.0
    out = packed_qkv_self_attention(mixed, d ** -0.5, causal=causal, bias=bias, dropout_p=0.1, seed=3, offset=9)
    m2 = mixed.detach().clone().requires_grad_(True)
    q, k, v = (m2[..., i * d:(i + 1) * d].permute(1, 0, 2, 3) for i in range(3))
    ref = flash_attn_func(q, k, v, dropout_p=0.1, softmax_scale=d ** -0.5, causal=causal, bias=bias, seed=3, offset=9)
    ref = ref.transpose(0, 1).reshape(s, b, h * d)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g)
    torch.testing.assert_close(mixed.grad, m2.grad, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_gpu_fused_vocab_cross_entropy(smoothing):
    """TP-1 fused CE (xentropy kernel on bf16 logits) vs fp32 Megatron-semantics math."""
    from apex.transformer.tensor_parallel.cross_entropy import _FusedCrossEntropy

    torch.manual_seed(1)
    s, b, v = 64, 4, 50304
    logits = (torch.randn(s, b, v, device="cuda") * 3).to(torch.bfloat16).requires_grad_(True)
    target = torch.randint(0, v, (s, b), device="cuda")
    loss = _FusedCrossEntropy.apply(logits, target, smoothing)
    x = logits.detach().float().requires_grad_(True)
    logp = torch.log_softmax(x, -1)
    nll = -logp.gather(-1, target.unsqueeze(-1)).squeeze(-1)
    if smoothing > 0:
        sm = smoothing * v / (v - 1)
        ref = (1 - sm) * nll - sm * logp.mean(-1)
    else:
        ref = nll
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    g = torch.rand_like(ref)
    loss.backward(g)
    ref.backward(g)
    torch.testing.assert_close(logits.grad.float(), x.grad, rtol=2e-2, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("with_bias", [True, False])
def test_gpu_fused_bias_dropout_add(with_bias):
    """gfx950 bias+dropout+residual kernel vs the torch mirror of the same counter-hash mask."""
    from apex.transformer.functional.fused_bias_dropout_add import _torch_bias_dropout_add, fused_bias_dropout_add

    torch.manual_seed(2)
    x = torch.randn(128, 4, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True)
    b = torch.randn(1024, device="cuda", dtype=torch.bfloat16, requires_grad=True) if with_bias else None
    y = fused_bias_dropout_add(x, b, r, 0.1, True, 77, 3)
    x2, r2 = (t.detach().float().requires_grad_(True) for t in (x, r))
    b2 = b.detach().float().requires_grad_(True) if with_bias else None
    ref = _torch_bias_dropout_add(x2, b2, r2, 0.1, 77, 3)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)
    g = torch.randn_like(ref)
    y.backward(g.to(y.dtype))
    ref.backward(g)
    torch.testing.assert_close(x.grad.float(), x2.grad, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(r.grad.float(), r2.grad, atol=1e-2, rtol=1e-2)
    if with_bias:
        torch.testing.assert_close(b.grad.float(), b2.grad, atol=0.5, rtol=2e-2)


def test_cpu_reference_functional_api_matches_modules():
    """The reference's functional module paths (``*_multihead_attn_func``) give the modules' results."""
    from apex.contrib.multihead_attn import EncdecMultiheadAttn, SelfMultiheadAttn
    from apex.contrib.multihead_attn.encdec_multihead_attn_func import encdec_attn_func
    from apex.contrib.multihead_attn.fast_encdec_multihead_attn_func import fast_encdec_attn_func
    from apex.contrib.multihead_attn.fast_self_multihead_attn_func import fast_self_attn_func
    from apex.contrib.multihead_attn.fast_self_multihead_attn_norm_add_func import fast_self_attn_norm_add_func
    from apex.contrib.multihead_attn.self_multihead_attn_func import SelfAttnFunc, self_attn_func

    torch.manual_seed(5)
    m = SelfMultiheadAttn(64, 4, bias=True, impl="default")
    x = torch.randn(10, 3, 64)
    kpm = torch.zeros(3, 10, dtype=torch.bool)
    kpm[2, 6:] = True
    ref, _ = m(x, x, x, key_padding_mask=kpm, is_training=False)
    got = self_attn_func(False, False, 4, m.scaling, x, m.in_proj_weight, m.out_proj_weight, m.in_proj_bias,
                         m.out_proj_bias, kpm, False, 0.0)
    torch.testing.assert_close(got, ref)
    assert SelfAttnFunc.apply is self_attn_func
    got = fast_self_attn_func(False, False, 4, x, m.in_proj_weight, m.out_proj_weight, m.in_proj_bias,
                              m.out_proj_bias, kpm, False, 0.0)
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-4)
    n = SelfMultiheadAttn(64, 4, include_norm_add=True, impl="fast")
    ref, _ = n(x, x, x, is_training=False)
    got = fast_self_attn_norm_add_func(False, False, 4, x, n.lyr_nrm_gamma_weights, n.lyr_nrm_beta_weights,
                                       n.in_proj_weight, n.out_proj_weight, None, 0.0)
    torch.testing.assert_close(got, ref)
    e = EncdecMultiheadAttn(64, 8, impl="default")
    q, kv = torch.randn(6, 2, 64), torch.randn(9, 2, 64)
    ref, _ = e(q, kv, kv, is_training=False)
    got = encdec_attn_func(False, False, 8, e.scaling, q, kv, e.in_proj_weight_q, e.in_proj_weight_kv,
                           e.out_proj_weight, None, None, None, None, 0.0)
    torch.testing.assert_close(got, ref)
    got = fast_encdec_attn_func(False, False, 8, q, kv, e.in_proj_weight_q, e.in_proj_weight_kv, e.out_proj_weight,
                                None, 0.0)
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("p", [0.0, 0.1, 0.25, 0.3333, 0.9])
def test_dropout_keep_scale_is_unbiased_for_the_16bit_threshold(p):
    from apex.ops.attention import dropout_keep_scale, dropout_keep_mask
    t16 = min(int(p * 65536.0), 65536)
    # exactly (65536 - t16) of the 65536 16-bit test values survive: scale x keep rate == 1
    assert dropout_keep_scale(p) * (65536 - t16) / 65536 == pytest.approx(1.0, rel=1e-12)
    keep = dropout_keep_mask(7, 0, [0, 1], 64, 256, p)
    assert abs(keep.float().mean().item() * dropout_keep_scale(p) - 1.0) < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("per_query", [False, True])
def test_gpu_flash_bias_vector_loads_bitwise(per_query):
    """The additive bias read as 16-byte key runs (key-contiguous bias over whole 64-key tiles) and
    as one value per key for a key-only bias in dK/dV: bitwise the per-element loads they replace,
    forced here by handing the same values in through a stride-2 view."""
    torch.manual_seed(21)
    b, s, h, d = 2, 256, 4, 64
    q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True)
    v = torch.randn_like(q, requires_grad=True)
    shape = (b, h, s, s) if per_query else (b, 1, 1, s)
    dense = torch.randn(*shape, device="cuda")
    dense[..., -s // 8:] = -10000.0
    wide = torch.zeros(*shape[:-1], 2 * s, device="cuda")
    wide[..., ::2] = dense
    strided = wide[..., ::2]
    assert strided.stride(-1) == 2 and torch.equal(strided, dense)
    g = torch.randn_like(q)
    outs = []
    for bias in (dense, strided):
        o = flash_attn_func(q, k, v, dropout_p=0.1, bias=bias, seed=5, offset=3)
        outs.append((o,) + torch.autograd.grad(o, (q, k, v), g))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
