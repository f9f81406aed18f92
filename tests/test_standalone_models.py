"""Standalone Megatron GPT / BERT over apex.transformer (reference
tests/L0/run_transformer/run_gpt_minimal_test.py and run_bert_minimal_test.py: build the model
with the TP/PP helpers, run forward/backward steps).  CPU tier: gloo world 2 — the TP=2 loss
must equal the TP=1 loss of the same (CPU-initialised) weights."""
import pytest
import torch

from tests._dist_utils import run_multiprocess


def _args(extra=()):
    return ["--num-layers", "2", "--hidden-size", "64", "--num-attention-heads", "4", "--seq-length", "16",
            "--max-position-embeddings", "16", "--micro-batch-size", "2", "--vocab-size", "128",
            "--use-cpu-initialization", "--hidden-dropout", "0", "--attention-dropout", "0",
            "--make-vocab-size-divisible-by", "8"] + list(extra)


def _build_and_loss(kind, tp, world):
    from apex.transformer import parallel_state
    from apex.transformer.testing import global_vars
    from apex.transformer.testing.standalone_bert import bert_model_provider
    from apex.transformer.testing.standalone_gpt import gpt_model_provider

    global_vars.destroy_global_vars()
    args = global_vars.set_global_variables(argv=_args(["--tensor-model-parallel-size", str(tp)]))
    if parallel_state.model_parallel_is_initialized():
        parallel_state.destroy_model_parallel()
    parallel_state.initialize_model_parallel(tp, 1)
    torch.manual_seed(123)
    g = torch.Generator().manual_seed(7)
    tokens = torch.randint(0, 100, (2, 16), generator=g)
    labels = torch.randint(0, 100, (2, 16), generator=g)
    if kind == "gpt":
        model = gpt_model_provider()
        pos = torch.arange(16).unsqueeze(0).expand(2, 16)
        loss = model(tokens, pos, None, labels=labels)
    else:
        model = bert_model_provider()
        mask = torch.ones(2, 16)
        mask[1, 12:] = 0
        loss, binary = model(tokens, mask, tokentype_ids=torch.zeros_like(tokens), lm_labels=labels)
        assert binary.shape == (2, 2)
    assert loss.shape == (2, 16)
    total = loss.mean() + (binary.float() ** 2).mean() if kind == "bert" else loss.mean()
    total.backward()
    grads_ok = all(p.grad is not None for p in model.parameters() if p.requires_grad)
    assert args.padded_vocab_size % (8 * tp) == 0
    return float(total), grads_ok


def _worker(rank, world, kind):
    l2, ok2 = _build_and_loss(kind, 2, world)
    l1, ok1 = _build_and_loss(kind, 1, world)
    assert ok1 and ok2
    assert abs(l1 - l2) < 1e-4 * max(1.0, abs(l1)), (l1, l2)


def test_gpt_tp2_matches_tp1():
    run_multiprocess(_worker, world=2, args=("gpt",))


def test_bert_tp2_matches_tp1():
    run_multiprocess(_worker, world=2, args=("bert",))


def test_arguments_derivations():
    from apex.transformer.testing.arguments import parse_args

    a = parse_args(argv=["--num-layers", "4", "--hidden-size", "256", "--num-attention-heads", "8", "--seq-length",
                         "32", "--vocab-size", "1000", "--bf16", "--micro-batch-size", "4"])
    assert a.ffn_hidden_size == 1024 and a.kv_channels == 32 and a.params_dtype == torch.bfloat16
    assert a.padded_vocab_size == 1024 and a.global_batch_size == 4 and a.encoder_seq_length == 32


def test_resnet_channels_last_global_pool_matches_adaptive_avgpool():
    """The fused-BN ResNet's global pool (models/resnet.py _SpatialMeanNHWC): same value and input
    gradient as flatten(AdaptiveAvgPool2d(1)), the gradient already in channels_last memory."""
    from apex.models.resnet import _SpatialMeanNHWC

    torch.manual_seed(0)
    x = torch.randn(3, 16, 7, 5, dtype=torch.float64).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = _SpatialMeanNHWC.apply(x)
    g = torch.randn_like(y)
    y.backward(g)
    x2 = x.detach().clone().requires_grad_()
    y2 = torch.flatten(torch.nn.AdaptiveAvgPool2d(1)(x2), 1)
    y2.backward(g)
    torch.testing.assert_close(y, y2)
    torch.testing.assert_close(x.grad, x2.grad)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,h,w", [(4, 2048, 7, 7), (3, 64, 5, 9)])
def test_gpu_global_pool_gradient_broadcast_is_bitwise_the_expand(n, c, h, w):
    """layout.hip spatial_broadcast (the pool's backward on the GPU) == the torch expand path."""
    from apex import _native

    ext = _native.require("conv").conv
    g = torch.randn(n, c, device="cuda").to(torch.bfloat16)
    got = ext.spatial_broadcast(g, h, w, 1.0 / (h * w))
    want = (g * (1.0 / (h * w))).view(n, 1, 1, c).expand(n, h, w, c).contiguous().permute(0, 3, 1, 2)
    assert got.is_contiguous(memory_format=torch.channels_last) and torch.equal(got, want)
