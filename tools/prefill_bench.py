#!/usr/bin/env python3
"""Prefill throughput of one knight turn (Llama-3-8B bf16, random init) on one GPU.

    python tools/prefill_bench.py [--tokens 11000] [--chunk N] [--reps 3]

Times ``Engine.prefill`` of a fresh sequence of ``--tokens`` random ids (after one warm-up
prefill), and reports tokens/s and model TFLOP/s (2 x params per token + causal attention).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=11000)
    ap.add_argument("--chunk", type=int, default=None, help="override EngineConfig.prefill_chunk")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from theroundtaible_amd.engine import Engine, EngineConfig
    kw = dict(model=a.model, weights="random:0", device="cuda:0", max_kv_tokens=(a.reps + 2) * (a.tokens + 64))
    if a.chunk:
        kw["prefill_chunk"] = a.chunk
    e = Engine(EngineConfig(**kw))
    cfg = e.cfg
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(5, cfg.vocab - 5, (a.tokens,), generator=g).tolist()
    e.prefill([(e.kv.seq("warm"), ids[:2048])])
    torch.cuda.synchronize()
    best = float("inf")
    for r in range(a.reps):
        s = e.kv.seq(f"r{r}")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.prefill([(s, ids)])
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
        e.release(f"r{r}")
    params = sum(t.numel() for t in e.model.w.values()) if hasattr(e.model, "w") else 0
    T = a.tokens
    attn_flops = 2 * 2 * cfg.n_layers * cfg.n_heads * cfg.head_dim * T * (T + 1) / 2
    gemm_flops = 2 * (params - 2 * cfg.vocab * cfg.hidden) * T   # embedding gather + last-row lm_head excluded
    print(json.dumps({"model": a.model, "tokens": T, "chunk": e.ecfg.prefill_chunk, "prefill_ms": round(best * 1e3, 1),
                      "tokens_per_s": round(T / best), "tflops": round((attn_flops + gemm_flops) / best / 1e12, 1)}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
