#!/usr/bin/env python3
"""Experiment: does warming the next GEMM's weights into the MALL on a side stream, during
the latency-bound decode attention, shorten (attention -> o-proj)?

Prints µs per (attention + o-proj) pair for: sequential; side-stream prefetch of W_o with
{16, 32, 64} workgroups; plus o-proj alone cold vs MALL-warm.
"""
from __future__ import annotations

import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from theroundtaible_amd import ops  # noqa: E402

DEV = "cuda"


def bf(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).to(torch.bfloat16)


def graph_time(body, iters=16, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            body(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            body(i)
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / iters)
    return best


def main():
    B, ctx, hq, hkv, d, hid = 3, 6000, 32, 8, 128, 4096
    nat = ops.native()
    copies = 24
    Wo = [ops.shuffle_weight(bf(hid, hq * d, scale=0.02)) for _ in range(copies)]
    nblk = (ctx + 31) // 32
    caches = [(bf(B * nblk, hkv, 32, d), bf(B * nblk, hkv, d, 32)) for _ in range(8)]
    bt = torch.arange(B * nblk, device=DEV, dtype=torch.int32).reshape(B, nblk)
    cl = torch.full((B,), ctx, device=DEV, dtype=torch.int32)
    q = bf(B, hq, d)
    splits = ops.decode_splits(B, hkv)
    ws = ops.DecodeWorkspace(B, hq, d, splits, DEV)
    out = torch.empty_like(q)
    res = bf(B, hid)
    sink = torch.zeros(1, dtype=torch.int32, device=DEV)
    side = torch.cuda.Stream()

    def attn(i):
        kc, vc = caches[i % 8]
        ops.paged_attention_decode(q, kc, vc, bt, cl, 1 / math.sqrt(d), splits, ws, out)

    def oproj(i, w=None):
        ops.skinny_gemm(out.reshape(B, -1), w if w is not None else Wo[i % copies], ops.PRO_PLAIN, ops.EPI_RESID,
                        res=res)

    print(f"o-proj cold            {graph_time(lambda i: oproj(i)):8.2f} us")
    print(f"o-proj MALL-warm       {graph_time(lambda i: oproj(i, Wo[0])):8.2f} us")
    print(f"attention alone        {graph_time(attn):8.2f} us")
    print(f"attn + o-proj seq      {graph_time(lambda i: (attn(i), oproj(i))):8.2f} us")
    for nwg in (8, 16, 32, 64):
        def body(i, nwg=nwg):
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                nat.prefetch(Wo[i % copies], nwg, sink)
            attn(i)
            cur.wait_stream(side)
            oproj(i)
        print(f"attn + o-proj, prefetch nwg={nwg:3d}  {graph_time(body):8.2f} us")


if __name__ == "__main__":
    main()
