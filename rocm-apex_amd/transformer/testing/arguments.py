"""Megatron-style command line arguments for the standalone test models
(reference apex/transformer/testing/arguments.py:21-806).

The flags are declared as data (group -> [(flag, kwargs)]) and validated / derived in
``_post_process`` (params dtype, kv channels, ffn size, padded vocab, data-parallel size,
global batch, virtual pipeline size, ...).  Usage:
``args = parse_args(extra_args_provider=None, defaults={}, override_args={}, ignore_unknown_args=False)``."""
import argparse
import os

import torch

_T = True
FLAGS = {
    "network size": [
        ("--num-layers", dict(type=int, default=None)), ("--hidden-size", dict(type=int, default=None)),
        ("--ffn-hidden-size", dict(type=int, default=None)), ("--num-attention-heads", dict(type=int, default=None)),
        ("--kv-channels", dict(type=int, default=None)), ("--max-position-embeddings", dict(type=int, default=None)),
        ("--make-vocab-size-divisible-by", dict(type=int, default=128)),
        ("--layernorm-epsilon", dict(type=float, default=1e-5)),
        ("--apply-residual-connection-post-layernorm", dict(action="store_true")),
        ("--openai-gelu", dict(action="store_true")), ("--onnx-safe", dict(type=bool, required=False)),
        ("--bert-no-binary-head", dict(action="store_false", dest="bert_binary_head")),
        ("--num-query-groups", dict(type=int, default=None)),
    ],
    "logging": [
        ("--log-params-norm", dict(action="store_true")), ("--log-num-zeros-in-grad", dict(action="store_true")),
        ("--tensorboard-log-interval", dict(type=int, default=1)),
        ("--tensorboard-queue-size", dict(type=int, default=1000)),
        ("--log-timers-to-tensorboard", dict(action="store_true")),
        ("--log-batch-size-to-tensorboard", dict(action="store_true")),
        ("--no-log-learnig-rate-to-tensorboard", dict(action="store_false", dest="log_learning_rate_to_tensorboard")),
        ("--no-log-loss-scale-to-tensorboard", dict(action="store_false", dest="log_loss_scale_to_tensorboard")),
        ("--log-validation-ppl-to-tensorboard", dict(action="store_true")),
        ("--log-memory-to-tensorboard", dict(action="store_true")),
    ],
    "regularization": [
        ("--attention-dropout", dict(type=float, default=0.1)), ("--hidden-dropout", dict(type=float, default=0.1)),
        ("--weight-decay", dict(type=float, default=0.01)), ("--clip-grad", dict(type=float, default=1.0)),
        ("--adam-beta1", dict(type=float, default=0.9)), ("--adam-beta2", dict(type=float, default=0.999)),
        ("--adam-eps", dict(type=float, default=1e-8)), ("--sgd-momentum", dict(type=float, default=0.9)),
    ],
    "training": [
        ("--micro-batch-size", dict(type=int, default=None)), ("--batch-size", dict(type=int, default=None)),
        ("--global-batch-size", dict(type=int, default=None)), ("--rampup-batch-size", dict(nargs="*", default=None)),
        ("--checkpoint-activations", dict(action="store_true")),
        ("--distribute-checkpointed-activations", dict(action="store_true")),
        ("--activations-checkpoint-method", dict(type=str, default=None, choices=["uniform", "block"])),
        ("--activations-checkpoint-num-layers", dict(type=int, default=1)),
        ("--train-iters", dict(type=int, default=None)), ("--train-samples", dict(type=int, default=None)),
        ("--log-interval", dict(type=int, default=100)), ("--exit-interval", dict(type=int, default=None)),
        ("--exit-duration-in-mins", dict(type=int, default=None)), ("--tensorboard-dir", dict(type=str, default=None)),
        ("--no-masked-softmax-fusion", dict(action="store_false", dest="masked_softmax_fusion")),
        ("--no-bias-gelu-fusion", dict(action="store_false", dest="bias_gelu_fusion")),
        ("--no-bias-dropout-fusion", dict(action="store_false", dest="bias_dropout_fusion")),
        ("--optimizer", dict(type=str, default="adam", choices=["adam", "sgd"])),
        ("--dataloader-type", dict(type=str, default=None, choices=["single", "cyclic"])),
        ("--no-async-tensor-model-parallel-allreduce",
         dict(action="store_true")),
        ("--sequence-parallel", dict(action="store_true")),
        ("--no-flash-attention", dict(action="store_false", dest="use_flash_attention")),
    ],
    "initialization": [
        ("--seed", dict(type=int, default=1234)), ("--init-method-std", dict(type=float, default=0.02)),
        ("--init-method-xavier-uniform", dict(action="store_true")),
    ],
    "learning rate": [
        ("--lr", dict(type=float, default=None)),
        ("--lr-decay-style", dict(type=str, default="linear", choices=["constant", "linear", "cosine"])),
        ("--lr-decay-iters", dict(type=int, default=None)), ("--lr-decay-samples", dict(type=int, default=None)),
        ("--lr-warmup-fraction", dict(type=float, default=None)), ("--lr-warmup-iters", dict(type=int, default=0)),
        ("--lr-warmup-samples", dict(type=int, default=0)), ("--warmup", dict(type=int, default=None)),
        ("--min-lr", dict(type=float, default=0.0)), ("--override-lr-scheduler", dict(action="store_true")),
        ("--use-checkpoint-lr-scheduler", dict(action="store_true")),
    ],
    "checkpointing": [
        ("--save", dict(type=str, default=None)), ("--save-interval", dict(type=int, default=None)),
        ("--no-save-optim", dict(action="store_true", default=None)),
        ("--no-save-rng", dict(action="store_true", default=None)), ("--load", dict(type=str, default=None)),
        ("--no-load-optim", dict(action="store_true", default=None)),
        ("--no-load-rng", dict(action="store_true", default=None)), ("--finetune", dict(action="store_true")),
    ],
    "mixed precision": [
        ("--fp16", dict(action="store_true")), ("--bf16", dict(action="store_true")),
        ("--loss-scale", dict(type=float, default=None)), ("--initial-loss-scale", dict(type=float, default=2 ** 32)),
        ("--min-loss-scale", dict(type=float, default=1.0)), ("--loss-scale-window", dict(type=float, default=1000)),
        ("--hysteresis", dict(type=int, default=2)), ("--fp32-residual-connection", dict(action="store_true")),
        ("--no-query-key-layer-scaling", dict(action="store_false", dest="apply_query_key_layer_scaling")),
        ("--attention-softmax-in-fp32", dict(action="store_true")),
        ("--accumulate-allreduce-grads-in-fp32", dict(action="store_true")),
        ("--fp16-lm-cross-entropy", dict(action="store_true")),
    ],
    "distributed": [
        ("--tensor-model-parallel-size", dict(type=int, default=1)),
        ("--pipeline-model-parallel-size", dict(type=int, default=1)),
        ("--pipeline-model-parallel-split-rank", dict(type=int, default=None)),
        ("--model-parallel-size", dict(type=int, default=None)),
        ("--num-layers-per-virtual-pipeline-stage", dict(type=int, default=None)),
        ("--distributed-backend", dict(default="nccl", choices=["nccl", "gloo"])),
        ("--DDP-impl", dict(default="local", choices=["local", "torch"])),
        ("--no-contiguous-buffers-in-local-ddp", dict(action="store_false", dest="use_contiguous_buffers_in_local_ddp")),
        ("--no-scatter-gather-tensors-in-pipeline", dict(action="store_false", dest="scatter_gather_tensors_in_pipeline")),
        ("--local_rank", dict(type=int, default=None)), ("--lazy-mpu-init", dict(type=bool, required=False)),
        ("--use-cpu-initialization", dict(action="store_true", default=None)),
        ("--empty-unused-memory-level", dict(default=0, type=int, choices=[0, 1, 2])),
    ],
    "validation": [
        ("--eval-iters", dict(type=int, default=100)), ("--eval-interval", dict(type=int, default=1000)),
    ],
    "data and dataloader": [
        ("--data-path", dict(nargs="*", default=None)), ("--split", dict(type=str, default="969, 30, 1")),
        ("--vocab-file", dict(type=str, default=None)), ("--merge-file", dict(type=str, default=None)),
        ("--vocab-extra-ids", dict(type=int, default=0)), ("--seq-length", dict(type=int, default=None)),
        ("--encoder-seq-length", dict(type=int, default=None)), ("--decoder-seq-length", dict(type=int, default=None)),
        ("--retriever-seq-length", dict(type=int, default=256)), ("--sample-rate", dict(type=float, default=1.0)),
        ("--mask-prob", dict(type=float, default=0.15)), ("--short-seq-prob", dict(type=float, default=0.1)),
        ("--mmap-warmup", dict(action="store_true")), ("--num-workers", dict(type=int, default=2)),
        ("--tokenizer-type", dict(type=str, default=None)), ("--data-impl", dict(type=str, default="infer")),
        ("--reset-position-ids", dict(action="store_true")), ("--reset-attention-mask", dict(action="store_true")),
        ("--eod-mask-loss", dict(action="store_true")), ("--padded-vocab-size", dict(type=int, default=None)),
        ("--vocab-size", dict(type=int, default=None)),
    ],
    "autoresume": [
        ("--adlr-autoresume", dict(action="store_true")), ("--adlr-autoresume-interval", dict(type=int, default=1000)),
    ],
}


def build_parser(extra_args_provider=None):
    parser = argparse.ArgumentParser(description="Megatron-LM arguments (apex standalone models)", allow_abbrev=False)
    for title, flags in FLAGS.items():
        g = parser.add_argument_group(title=title)
        for flag, kw in flags:
            g.add_argument(flag, **kw)
    if extra_args_provider is not None:
        parser = extra_args_provider(parser)
    return parser


def _post_process(args, defaults):
    args.rank = int(os.getenv("RANK", "0"))
    args.world_size = int(os.getenv("WORLD_SIZE", "1"))
    for k, v in defaults.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
    if args.model_parallel_size is not None:
        args.tensor_model_parallel_size = args.model_parallel_size
    args.tensor_model_parallel_size = min(args.tensor_model_parallel_size, args.world_size)
    assert args.world_size % args.tensor_model_parallel_size == 0, "world size not divisible by TP size"
    args.pipeline_model_parallel_size = min(args.pipeline_model_parallel_size,
                                            args.world_size // args.tensor_model_parallel_size)
    mp = args.tensor_model_parallel_size * args.pipeline_model_parallel_size
    assert args.world_size % mp == 0, "world size not divisible by TP x PP"
    args.data_parallel_size = args.world_size // mp
    if args.batch_size is not None:
        args.micro_batch_size = args.micro_batch_size or args.batch_size
    if args.global_batch_size is None and args.micro_batch_size is not None:
        args.global_batch_size = args.micro_batch_size * args.data_parallel_size
    if args.num_layers_per_virtual_pipeline_stage is not None:
        assert args.pipeline_model_parallel_size > 2, "virtual pipeline needs pipeline size > 2"
        assert args.num_layers % args.num_layers_per_virtual_pipeline_stage == 0
        args.virtual_pipeline_model_parallel_size = (args.num_layers // args.pipeline_model_parallel_size) // \
            args.num_layers_per_virtual_pipeline_stage
    else:
        args.virtual_pipeline_model_parallel_size = None
    args.params_dtype = torch.float
    if args.fp16:
        assert not args.bf16, "--fp16 and --bf16 are exclusive"
        args.params_dtype = torch.half
    if args.bf16:
        args.params_dtype = torch.bfloat16
        args.accumulate_allreduce_grads_in_fp32 = True
    if args.fp16 or args.bf16:
        args.apply_query_key_layer_scaling = args.apply_query_key_layer_scaling and args.fp16
    if args.ffn_hidden_size is None and args.hidden_size is not None:
        args.ffn_hidden_size = 4 * args.hidden_size
    if args.kv_channels is None and args.hidden_size is not None and args.num_attention_heads:
        assert args.hidden_size % args.num_attention_heads == 0
        args.kv_channels = args.hidden_size // args.num_attention_heads
    if args.seq_length is not None and args.encoder_seq_length is None:
        args.encoder_seq_length = args.seq_length
    elif args.encoder_seq_length is not None and args.seq_length is None:
        args.seq_length = args.encoder_seq_length
    if args.seq_length is not None and args.max_position_embeddings is not None:
        assert args.max_position_embeddings >= args.seq_length
    if args.padded_vocab_size is None and args.vocab_size is not None:
        mult = args.make_vocab_size_divisible_by * args.tensor_model_parallel_size
        args.padded_vocab_size = ((args.vocab_size + mult - 1) // mult) * mult
    if args.lr is not None:
        assert args.min_lr <= args.lr
    if args.save is not None:
        assert args.save_interval is not None
    if args.use_cpu_initialization is None:
        args.use_cpu_initialization = not torch.cuda.is_available()
    if args.activations_checkpoint_method is None and args.checkpoint_activations:
        args.activations_checkpoint_method = "uniform"
    if args.sequence_parallel and args.tensor_model_parallel_size == 1:
        args.sequence_parallel = False
    if args.num_query_groups is None:
        args.num_query_groups = args.num_attention_heads
    return args


def parse_args(extra_args_provider=None, defaults=None, override_args=None, ignore_unknown_args=False, argv=None):
    parser = build_parser(extra_args_provider)
    if ignore_unknown_args:
        args, _ = parser.parse_known_args(argv)
    else:
        args = parser.parse_args(argv)
    for k, v in (override_args or {}).items():
        setattr(args, k, v)
    return _post_process(args, defaults or {})
