#!/usr/bin/env python3
"""Standalone Megatron GPT (apex.transformer.testing) forward/backward on one MI355X, bf16,
flash attention, TP=1 — prints loss and step time.  Run: python tools/gpu_gpt_smoke.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")

import torch  # noqa: E402


def main():
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", rank=0, world_size=1)
    from apex.optimizers import FusedAdam
    from apex.transformer import parallel_state
    from apex.transformer.testing import global_vars
    from apex.transformer.testing.standalone_gpt import gpt_model_provider

    global_vars.set_global_variables(argv=[
        "--num-layers", "12", "--hidden-size", "1024", "--num-attention-heads", "16", "--seq-length", "2048",
        "--max-position-embeddings", "2048", "--micro-batch-size", "4", "--vocab-size", "50304", "--bf16",
        "--hidden-dropout", "0.1", "--attention-dropout", "0.1"])
    parallel_state.initialize_model_parallel(1, 1)
    from apex.transformer import tensor_parallel

    tensor_parallel.model_parallel_cuda_manual_seed(1234)
    model = gpt_model_provider()
    opt = FusedAdam(model.parameters(), lr=1e-4)
    tokens = torch.randint(0, 50304, (4, 2048), device="cuda")
    pos = torch.arange(2048, device="cuda").unsqueeze(0).expand(4, -1)
    labels = torch.randint(0, 50304, (4, 2048), device="cuda")

    def step():
        loss = model(tokens, pos, None, labels=labels).float().mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(3):
        loss = step()
    torch.cuda.synchronize()
    t = time.time()
    n = 10
    for _ in range(n):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.time() - t) / n
    ntok = 4 * 2048
    params = sum(p.numel() for p in model.parameters())
    flops = 6 * params * ntok + 12 * 12 * 1024 * 2048 * ntok  # dense + attention (causal counted full)
    print("gpt345m bf16 flash: loss {:.4f}  step {:.1f} ms  {:.0f} tokens/s  ~{:.0f} TFLOP/s".format(
        float(loss), dt * 1e3, ntok / dt, flops / dt / 1e12), flush=True)
    assert torch.isfinite(loss)


if __name__ == "__main__":
    main()
