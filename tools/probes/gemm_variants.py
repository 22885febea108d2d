#!/usr/bin/env python3
"""Probe: where the fixed cost of a tensor-parallel shard GEMM goes. Times the decode GEMM of one
shard shape with each prologue / epilogue combination (PLAIN / NORM / NORM_ADD x STORE / ROPE /
SWIGLU) so the cost of each piece of fused work can be read off against the pure weight stream
(tools/probes/stream_probe.hip). Same harness as tools/microbench.py (hipGraph of 20 calls,
>= 1 GiB of rotating weight copies, so every call reads cold weights).

    python tools/probes/gemm_variants.py [--tp 2,8]
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from microbench import bf, timed  # noqa: E402
from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.ops import reference as ref  # noqa: E402

DEV = "cuda"


def run(tp: int, M: int = 3):
    hid, d, hq, hkv, ffn = 4096, 128, 32 // tp, max(1, 8 // tp), 14336 // tp
    x, x2, xo = bf(M, hid), bf(M, hid), bf(M, hid)
    nb = 64
    kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
    cs = ref.rope_cos_sin(8192, d, 500000.0, DEV)
    pos = torch.arange(M, device=DEV, dtype=torch.int64) + 100
    slots = torch.arange(M, device=DEV, dtype=torch.int64) + 40
    sw = ops.split_workspace(DEV)
    for label, sk in (("split-K ws", dict(split_ws=sw, split_mode=ops.SPLIT_K)), ("no ws", {})):
        N, K = (hq + 2 * hkv) * d, hid
        copies = max(2, math.ceil(2**30 / (N * K * 2)))
        Ws = [ops.shuffle_weight(bf(N, K, scale=0.02), rope_heads=hq + hkv, head_dim=d) for _ in range(copies)]
        cases = {
            "plain/store": lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_PLAIN, ops.EPI_STORE, **sk),
            "norm/store": lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM, ops.EPI_STORE, **sk),
            "norm_add/store": lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM_ADD, ops.EPI_STORE, x2=x2,
                                                        xout=xo, **sk),
            "norm/rope": lambda i: ops.skinny_gemm_rope(x, Ws[i % copies], ops.PRO_NORM, pos, cs, kc, vc, slots, hq,
                                                        hkv, d, **sk),
            "norm_add/rope": lambda i: ops.skinny_gemm_rope(x, Ws[i % copies], ops.PRO_NORM_ADD, pos, cs, kc, vc,
                                                            slots, hq, hkv, d, x2=x2, xout=xo, **sk),
        }
        for name, fn in cases.items():
            print(f"tp{tp} qkv N={N} K={K} {label:10s} {name:16s} {timed(fn):7.2f} us", flush=True)
        del Ws
        N = 2 * ffn
        copies = max(2, math.ceil(2**30 / (N * K * 2)))
        Ws = [ops.shuffle_weight(bf(N, K, scale=0.02), swiglu=True) for _ in range(copies)]
        cases = {
            "plain/swiglu": lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_PLAIN, ops.EPI_SWIGLU, **sk),
            "norm/swiglu": lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM, ops.EPI_SWIGLU, **sk),
            "norm_add/swiglu": lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM_ADD, ops.EPI_SWIGLU, x2=x2,
                                                         xout=xo, **sk),
        }
        for name, fn in cases.items():
            print(f"tp{tp} gate_up N={N} K={K} {label:10s} {name:16s} {timed(fn):7.2f} us", flush=True)
        del Ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", default="2,8")
    a = ap.parse_args()
    torch.manual_seed(0)
    for t in a.tp.split(","):
        run(int(t))
