"""Transformer training benchmarks of BASELINE.json (configs 4 and 5), driven by ``bench.py --model``:

* ``gpt2-medium``: Megatron GPT (apex.transformer.testing.standalone_gpt) 24 x 1024, 16 heads,
  seq 1024, vocab 50257 (padded to 50304), amp O2 bf16 + FusedAdam; the MLP runs as the fused
  GEMM+bias+GeLU -> GEMM pair (apex.fused_dense kernels), attention as the gfx950 flash kernel.
  Metric: tokens/s for the whole job.
* ``bert-large``: Megatron BERT 24 x 1024, 16 heads, seq 512, vocab 30522, NSP head, amp O2 bf16
  + FusedLAMB (multi_tensor_lamb + l2norm).  Metric: sequences/s for the whole job.

Data parallel over every rank (TP = PP = 1) with apex.parallel.DistributedDataParallel; synthetic
token ids / labels resident on the GPU; random-init weights (no checkpoints, no network)."""
import torch
import torch.distributed as dist

CONFIGS = {
    "gpt2-medium": dict(layers=24, hidden=1024, heads=16, seq=1024, vocab=50257, micro_batch=16, kind="gpt"),
    "bert-large": dict(layers=24, hidden=1024, heads=16, seq=512, vocab=30522, micro_batch=32, kind="bert"),
}


def _ensure_process_group():
    if not dist.is_initialized():  # single GPU: a one-rank group (parallel_state needs one)
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)


def build(args, dev, distributed):
    import apex
    from apex import amp
    from apex.optimizers import FusedAdam, FusedLAMB
    from apex.transformer import parallel_state, tensor_parallel
    from apex.transformer.testing import global_vars

    cfg = CONFIGS[args.model]
    B = args.batch_size if args.batch_size_set else cfg["micro_batch"]
    S = cfg["seq"]
    _ensure_process_group()
    global_vars.destroy_global_vars()
    global_vars.set_global_variables(argv=[
        "--num-layers", str(cfg["layers"]), "--hidden-size", str(cfg["hidden"]),
        "--num-attention-heads", str(cfg["heads"]), "--seq-length", str(S),
        "--max-position-embeddings", str(S), "--micro-batch-size", str(B), "--vocab-size", str(cfg["vocab"]),
        "--hidden-dropout", "0.1", "--attention-dropout", "0.1"])
    parallel_state.destroy_model_parallel()
    parallel_state.initialize_model_parallel(1, 1)
    tensor_parallel.model_parallel_cuda_manual_seed(1234)
    if cfg["kind"] == "gpt":
        from apex.transformer.testing.standalone_gpt import gpt_model_provider as provider
    else:
        from apex.transformer.testing.standalone_bert import bert_model_provider as provider
    model = provider().to(dev)
    low = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    # fused amp (as the headline ResNet bench): the optimizer kernel reads the bf16 model grads with
    # the device inverse loss scale -- no fp32 master-grad materialization pass and no per-parameter
    # zero fill of the model grads (--materialize-master-grads: the reference-style path)
    mm = bool(getattr(args, "materialize_master_grads", False))
    if cfg["kind"] == "gpt":
        opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01, materialize_master_grads=mm)
    else:
        opt = FusedLAMB(model.parameters(), lr=1e-4, weight_decay=0.01, max_grad_norm=1.0, materialize_master_grads=mm)
    model, opt = amp.initialize(model, opt, opt_level=args.opt_level, cast_model_type=low, verbosity=0)
    if distributed:
        model = apex.parallel.DistributedDataParallel(model, message_size=int(getattr(args, "message_size", 1e7)))
    V = cfg["vocab"]
    tokens = torch.randint(0, V, (B, S), device=dev)
    labels = torch.randint(0, V, (B, S), device=dev)
    if cfg["kind"] == "gpt":
        pos = torch.arange(S, device=dev).unsqueeze(0).expand(B, -1)

        def loss_fn():
            return model(tokens, pos, None, labels=labels).float().mean()
    else:
        mask = torch.ones(B, S, device=dev)
        mask[::4, S * 3 // 4:] = 0  # some padded sequences
        types = torch.zeros(B, S, dtype=torch.long, device=dev)
        nsp = torch.randint(0, 2, (B,), device=dev)

        def loss_fn():
            lm_loss, binary_logits = model(tokens, mask, tokentype_ids=types, lm_labels=labels)
            return lm_loss.float().mean() + torch.nn.functional.cross_entropy(binary_logits.float(), nsp)

    # graph-safe dropout: the native dropout kernels read a device step counter that each step
    # advances on the device, so a hipGraph-captured step (bench.py --graph) draws fresh masks on
    # every replay (apex.ops.dropout_rng)
    from apex.ops import dropout_rng

    dropout_rng.enable()

    def step():
        dropout_rng.advance(dev)
        loss = loss_fn()
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        return loss

    params = sum(p.numel() for p in model.parameters())
    return step, B, S, params


def describe(args, B, S, world, params):
    cfg = CONFIGS[args.model]
    gpt = cfg["kind"] == "gpt"
    return {
        "metric": ("tokens/sec (whole job) GPT-2 medium amp O2 + fused_dense + FusedAdam" if gpt
                   else "sequences/sec (whole job) BERT-large seq512 amp O2 + FusedLAMB"),
        "unit": "tokens/s" if gpt else "sequences/s",
        "items_per_gpu_step": B * S if gpt else B,
        "config": {"model": args.model, "layers": cfg["layers"], "hidden": cfg["hidden"], "heads": cfg["heads"],
                   "params": params, "global_batch": B * world, "per_gpu_batch": B, "seq_len": S,
                   "opt_level": args.opt_level,
                   "optimizer": ("FusedAdam" if gpt else "FusedLAMB") + (
                       " (materialized fp32 master grads)" if getattr(args, "materialize_master_grads", False)
                       else " (fused amp: bf16 model grads -> fp32 master + bf16 model in one pass)"),
                   "attention": "gfx950 flash (causal)" if gpt else "gfx950 flash (key-padding bias)",
                   "parallelism": f"dp{world}"},
    }


def build_torch_baseline(args, dev, distributed):
    """Stock reference point for configs 4 / 5 on the same box: Hugging Face GPT-2 medium /
    BERT-large (random init, same sizes, seq, micro-batch and dropout 0.1) with PyTorch SDPA
    attention, torch.autocast bf16, torch.optim.AdamW(fused=True) / AdamW for BERT (torch has no
    LAMB), torch DDP.  ``bench.py --model gpt2-medium --impl torch``."""
    from transformers import BertConfig, BertForPreTraining, GPT2Config, GPT2LMHeadModel

    cfg = CONFIGS[args.model]
    B = args.batch_size if args.batch_size_set else cfg["micro_batch"]
    S = cfg["seq"]
    V = cfg["vocab"]
    if cfg["kind"] == "gpt":
        conf = GPT2Config(n_layer=cfg["layers"], n_embd=cfg["hidden"], n_head=cfg["heads"], n_positions=S,
                          vocab_size=V, resid_pdrop=0.1, embd_pdrop=0.1, attn_pdrop=0.1,
                          bos_token_id=V - 1, eos_token_id=V - 1, attn_implementation="sdpa")
        model = GPT2LMHeadModel(conf).to(dev)
    else:
        conf = BertConfig(num_hidden_layers=cfg["layers"], hidden_size=cfg["hidden"],
                          num_attention_heads=cfg["heads"], intermediate_size=4 * cfg["hidden"],
                          max_position_embeddings=S, vocab_size=V, hidden_dropout_prob=0.1,
                          attention_probs_dropout_prob=0.1, attn_implementation="sdpa")
        model = BertForPreTraining(conf).to(dev)
    if distributed:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
    tokens = torch.randint(0, V, (B, S), device=dev)
    labels = torch.randint(0, V, (B, S), device=dev)
    if cfg["kind"] == "bert":
        mask = torch.ones(B, S, device=dev, dtype=torch.long)
        mask[::4, S * 3 // 4:] = 0
        nsp = torch.randint(0, 2, (B,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if cfg["kind"] == "gpt":
                loss = model(input_ids=tokens, labels=labels).loss
            else:
                loss = model(input_ids=tokens, attention_mask=mask, labels=labels, next_sentence_label=nsp).loss
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    params = sum(p.numel() for p in model.parameters())
    return step, B, S, params
