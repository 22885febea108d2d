"""Probe: how much of a round's prefill is host time at the tp 8 shard shapes?

One varlen prefill forward (the bench's per-round shape: ~1.8K new tokens over a long prefix) on
the Llama-3-8B tp 8 rank-0 shard model (hidden 4096, 4 / 1 heads, FFN 1792, 32 layers,
collectives elided as in ``bench.py --simulate-tp``): wall-clock (host, synchronised) vs the GPU
time between events around the same call; token counts change per call (as between rounds) or
repeat; hipBLASLt (torch default) vs rocBLAS for the prefill GEMMs.

    python tools/probes/prefill_host.py [--ctx 16384]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from theroundtaible_amd.engine import Engine, EngineConfig  # noqa: E402
from theroundtaible_amd.models import config as mcfg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=16384)
    ap.add_argument("--layers", type=int, default=32)
    a = ap.parse_args()
    mcfg.PRESETS["tp8shard"] = mcfg.ModelConfig("tp8shard", "llama", a.layers, 4096, 4, 1, 128, 1792, 128256 // 8,
                                                131072, 500000.0, 1e-5)
    nb = (a.ctx + 40 * 2048) // 32 + 64
    e = Engine(EngineConfig(model="tp8shard", weights="random-full:5", device="cuda", num_blocks=nb, use_graphs=False))
    g = torch.Generator().manual_seed(1)
    s = e.kv.seq("s")
    e.prefill([(s, torch.randint(0, 16032, (a.ctx,), generator=g).tolist())])
    torch.cuda.synchronize()
    rows = []
    for lib in ("default", "rocblas"):
        if lib == "rocblas":
            torch.backends.cuda.preferred_blas_library("cublas")
        for i, T in enumerate([1772, 1790, 1745, 1772, 1772, 1801, 1763]):
            ids = torch.randint(0, 16032, (T,), generator=g).tolist()
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            ev0.record()
            e.prefill([(s, ids)])
            ev1.record()
            t_launch = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            row = {"blas": lib, "T": T, "wall_ms": round((t1 - t0) * 1e3, 2),
                   "host_enqueue_ms": round((t_launch - t0) * 1e3, 2), "gpu_ms": round(ev0.elapsed_time(ev1), 2)}
            rows.append(row)
            print(json.dumps(row), flush=True)
            e.kv.truncate(s, a.ctx)
    torch.backends.cuda.preferred_blas_library("cublaslt")
    print(json.dumps({"rows": rows}))


if __name__ == "__main__":
    main()
