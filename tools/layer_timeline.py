#!/usr/bin/env python3
"""Phase timeline of the persistent decode-layer kernel on one Llama-3-8B-shaped layer.

Every workgroup stamps ``s_memrealtime`` (100 MHz) at each phase boundary; this prints the
median/max per phase over workgroups and the wall time of the launch, next to the same layer
as five separate launches (hipGraph-timed).

    python tools/layer_timeline.py [--batch 4] [--ctx 6000] [--splits 8]
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.ops import reference as ref  # noqa: E402

DEV = "cuda"
NAMES = ["P1 qkv", "wait qkv", "P2 attn", "wait attn", "P3 o", "wait o", "P4 gate_up", "wait gu", "P5 down"]


def bf(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).to(torch.bfloat16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--ctx", type=int, default=6000)
    ap.add_argument("--splits", type=int, default=8)
    a = ap.parse_args()
    B, ctx, S = a.batch, a.ctx, a.splits
    H, I, hq, hkv, D = 4096, 14336, 32, 8, 128
    gam = torch.ones(H, dtype=torch.bfloat16, device=DEV)
    lw = {"wqkv": ops.shuffle_weight(bf((hq + 2 * hkv) * D, H, scale=0.02), gam, rope_heads=hq + hkv, head_dim=D),
          "wo": ops.shuffle_weight(bf(H, hq * D, scale=0.02)),
          "w_gate_up": ops.shuffle_weight(bf(2 * I, H, scale=0.02), gam, swiglu=True),
          "w_down": ops.shuffle_weight(bf(H, I, scale=0.02))}
    nblk = (ctx + 32) // 32 + 1
    kc, vc = bf(B * nblk, hkv, 32, D), bf(B * nblk, hkv, D, 32)
    bt = torch.arange(B * nblk, device=DEV, dtype=torch.int32).reshape(B, nblk)
    pos = torch.full((B,), ctx, device=DEV, dtype=torch.int64)
    slots = (bt[:, ctx // 32].long() * 32 + ctx % 32)
    cl = (pos + 1).to(torch.int32)
    cs = ref.rope_cos_sin(ctx + 64, D, 500000.0, DEV)
    ws = ops.DecodeWorkspace(B, hq, D, S, DEV)
    res = bf(B, H)
    G = ops.native().decode_layer_grid()
    stamps = torch.zeros(G, 10, dtype=torch.int64, device=DEV)
    scale = 1 / math.sqrt(D)

    def persistent(st=None):
        ops.decode_layer(res, lw, pos, cs, kc, vc, slots, bt, cl, hq, hkv, D, S, ws, 1e-5, scale, stamps=st)

    for _ in range(3):
        persistent()
    torch.cuda.synchronize()
    rows = []
    for _ in range(5):
        persistent(stamps)
        torch.cuda.synchronize()
        t = stamps.double() * 10e-3   # 100 MHz ticks -> µs
        t0 = t[:, 0].min()
        d = t[:, 1:] - t[:, :-1]
        rows.append((d, float(t[:, 9].max() - t0)))
    assert int(ws.err.item()) == 0, "poll expired"
    d, wall = rows[-1]
    print(f"persistent layer: grid {G}, B={B}, ctx={ctx}, splits={S}: wall {wall:.1f} us (stamps)")
    for i, n in enumerate(NAMES):
        col = d[:, i]
        print(f"  {n:12s} median {col.median():7.2f}  max {col.max():7.2f} us")

    # same layer as 5 launches, graph-timed, and the persistent launch graph-timed
    q = torch.empty(B, hq, D, dtype=torch.bfloat16, device=DEV)

    def five():
        qq = ops.skinny_gemm_rope(res, lw["wqkv"], ops.PRO_NORM, pos, cs, kc, vc, slots, hq, hkv, D, 1e-5)
        att = ops.paged_attention_decode(qq, kc, vc, bt, cl, scale, S, ws)
        ops.skinny_gemm(att.reshape(B, -1), lw["wo"], ops.PRO_PLAIN, ops.EPI_RESID, res=res)
        g = ops.skinny_gemm(res, lw["w_gate_up"], ops.PRO_NORM, ops.EPI_SWIGLU, eps=1e-5)
        ops.skinny_gemm(g, lw["w_down"], ops.PRO_PLAIN, ops.EPI_RESID, res=res)

    for name, fn in (("five launches", five), ("persistent", persistent)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(8):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(4):
            gr.replay()
        ev1.record()
        torch.cuda.synchronize()
        print(f"{name:14s}: {ev0.elapsed_time(ev1) * 1000 / 32:7.1f} us per layer (hipGraph)")
    assert int(ws.err.item()) == 0


if __name__ == "__main__":
    main()
