#!/usr/bin/env python3
"""Multi-head attention latency at the reference's published configuration.

Capability / protocol of reference apex/contrib/examples/multihead_attn/perf_test_multihead_attn.py
:9-17 (the only numbers the reference publishes: apex/contrib/multihead_attn/README.md:54-60,
MHA_fwd.png / MHA_bwd.png, Titan V): a stack of ``--layers`` (18) self-attention layers, seq 64,
hidden 1024, 16 heads, dropout 0.1, fp16, no biases; ``--num-seqs`` sequences per batch
(10 -> 640 tokens, 120 -> 7680 tokens); forward and backward timed with device events over
``--trials`` after ``--warmup-trials``, reported per layer.

Implementations timed in ONE process on the same inputs (interleaved per batch size):
  fast    apex SelfMultiheadAttn(impl='fast')    — gfx950 flash-attention + MFMA GEMMs
  default apex SelfMultiheadAttn(impl='default') — the reference's python implementation path
  native  torch.nn.MultiheadAttention             — stock PyTorch-ROCm

Output: one JSON line per (impl, tokens) with fwd_ms / bwd_ms per layer, plus the published
Titan V values for the same row (read off the reference's charts).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

# published per-layer latencies (ms) on Titan V, BASELINE.md rows 25-31: impl -> tokens -> (fwd, bwd)
PUBLISHED = {
    "fast": {640: (0.20, 0.32), 7680: (1.02, 1.95)},
    "default": {640: (0.63, 0.89), 7680: (1.03, 2.03)},
    "native": {640: (0.90, 0.83), 7680: (1.52, 2.69)},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq-length", type=int, default=64)
    ap.add_argument("--num-seqs", type=int, nargs="+", default=[10, 120])
    ap.add_argument("--trials", type=int, default=20)
    ap.add_argument("--warmup-trials", type=int, default=5)
    ap.add_argument("--layers", type=int, default=18)
    ap.add_argument("--hidden-dim", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--impls", nargs="+", default=["fast", "default", "native"])
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--biases", action="store_true")
    ap.add_argument("--norm-add", action="store_true")
    ap.add_argument("--out", default=None, help="append the JSON lines to this file too")
    ap.add_argument("--graph", action="store_true",
                    help="also time the stack captured as two hipGraphs (forward, backward) per impl")
    return ap.parse_args()


def build(impl, a, dtype):
    from apex.contrib.multihead_attn import SelfMultiheadAttn

    layers = []
    for _ in range(a.layers):
        if impl == "native":
            m = torch.nn.MultiheadAttention(a.hidden_dim, a.heads, dropout=0.1, bias=a.biases)
        else:
            m = SelfMultiheadAttn(a.hidden_dim, a.heads, dropout=0.1, bias=a.biases, include_norm_add=a.norm_add,
                                  impl=impl)
        layers.append(m.cuda().to(dtype))
    return layers


def run_stack(impl, layers, x):
    h = x
    for m in layers:
        if impl == "native":
            h, _ = m(h, h, h, key_padding_mask=None, need_weights=False, attn_mask=None)
        else:
            h, _ = m(h, h, h, key_padding_mask=None, need_weights=False, attn_mask=None, is_training=True)
    return h


def time_impl(impl, layers, a, seqs, dtype):
    """Device time per layer (events) and the host's enqueue time per layer (wall clock of the
    python calls, GPU idle at the start of each trial): host >= device means launch-bound."""
    import time

    x = torch.randn(a.seq_length, seqs, a.hidden_dim, dtype=dtype, device="cuda").requires_grad_(True)
    g = torch.randn_like(x)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.trials)]
    host_f, host_b = [], []
    for t in range(a.warmup_trials + a.trials):
        i = t - a.warmup_trials
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if i >= 0:
            ev[i][0].record()
        out = run_stack(impl, layers, x)
        if i >= 0:
            ev[i][1].record()
        t1 = time.perf_counter()
        out.backward(g)
        if i >= 0:
            ev[i][2].record()
            host_f.append((t1 - t0) * 1e3 / a.layers)
            host_b.append((time.perf_counter() - t1) * 1e3 / a.layers)
        x.grad = None
        for m in layers:
            for p in m.parameters():
                p.grad = None
    torch.cuda.synchronize()
    fwd = sorted(e[0].elapsed_time(e[1]) / a.layers for e in ev)
    bwd = sorted(e[1].elapsed_time(e[2]) / a.layers for e in ev)
    return fwd, bwd, sorted(host_f)[len(host_f) // 2], sorted(host_b)[len(host_b) // 2]


def time_graph(impl, layers, a, seqs, dtype):
    """The same stack captured once as a forward and a backward hipGraph and replayed: the
    device-bound latency with the host launch cost removed (dropout stays graph-safe: the
    attention kernels read a device RNG step)."""
    x = torch.randn(a.seq_length, seqs, a.hidden_dim, dtype=dtype, device="cuda").requires_grad_(True)
    g = torch.randn_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            run_stack(impl, layers, x).backward(g)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gf, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf):
        out = run_stack(impl, layers, x)
    with torch.cuda.graph(gb, pool=gf.pool()):
        out.backward(g)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.trials)]
    for t in range(a.warmup_trials + a.trials):
        i = t - a.warmup_trials
        if i >= 0:
            ev[i][0].record()
        gf.replay()
        if i >= 0:
            ev[i][1].record()
        gb.replay()
        if i >= 0:
            ev[i][2].record()
    torch.cuda.synchronize()
    fwd = sorted(e[0].elapsed_time(e[1]) / a.layers for e in ev)
    bwd = sorted(e[1].elapsed_time(e[2]) / a.layers for e in ev)
    return fwd, bwd


def main():
    a = parse()
    if not torch.cuda.is_available():
        raise SystemExit("needs a GPU")
    torch.manual_seed(111)
    dtype = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    stacks = {impl: build(impl, a, dtype) for impl in a.impls}
    lines = []
    for seqs in a.num_seqs:
        tokens = seqs * a.seq_length
        runs = [(impl, False) for impl in a.impls] + ([(impl, True) for impl in a.impls if impl != "native"]
                                                        if a.graph else [])
        for impl, graphed in runs:
            host = None
            if graphed:
                fwd, bwd = time_graph(impl, stacks[impl], a, seqs, dtype)
            else:
                fwd, bwd, hf, hb = time_impl(impl, stacks[impl], a, seqs, dtype)
                host = (hf, hb)
            pub = PUBLISHED.get(impl, {}).get(tokens) if (a.seq_length == 64 and a.hidden_dim == 1024
                                                           and a.heads == 16 and a.layers == 18) else None
            med_f, med_b = fwd[len(fwd) // 2], bwd[len(bwd) // 2]
            rec = {"impl": impl + ("+graph" if graphed else ""), "tokens": tokens, "sequences": seqs, "seq_length": a.seq_length,
                   "hidden": a.hidden_dim, "heads": a.heads, "layers": a.layers, "dtype": a.dtype,
                   "dropout": 0.1, "biases": a.biases, "norm_add": a.norm_add,
                   "fwd_ms_per_layer": round(sum(fwd) / len(fwd), 4), "bwd_ms_per_layer": round(sum(bwd) / len(bwd), 4),
                   "fwd_ms_median": round(med_f, 4), "bwd_ms_median": round(med_b, 4),
                   "fwd_ms_min": round(fwd[0], 4), "bwd_ms_min": round(bwd[0], 4)}
            if host is not None:
                rec["host_enqueue_fwd_ms_per_layer"], rec["host_enqueue_bwd_ms_per_layer"] = round(host[0], 4), \
                    round(host[1], 4)
            if pub is not None:
                rec["published_titanv_fwd_ms"], rec["published_titanv_bwd_ms"] = pub
                rec["speedup_vs_published_fwd"] = round(pub[0] / rec["fwd_ms_per_layer"], 2)
                rec["speedup_vs_published_bwd"] = round(pub[1] / rec["bwd_ms_per_layer"], 2)
            print(json.dumps(rec), flush=True)
            lines.append(rec)
    if a.out:
        with open(a.out, "a") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
