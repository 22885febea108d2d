#!/usr/bin/env python3
"""Kernel microbenchmarks on the GPU: the decode hot ops of a Llama-3-8B knight batch.

Each op is captured N times into a hipGraph and replayed, so launch overhead does not
inflate the per-call time. Weight-streaming ops rotate over enough distinct copies
(>= 1 GiB) that the 256 MB MALL cannot serve repeats — matching a real decode step,
which streams all 16 GB of weights once. Prints one markdown table (µs, achieved TB/s).

    python tools/microbench.py [--batch 3] [--ctx 6000] [--only gemm,attn,sample,prefill]
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
ROWS = []


def timed(fn, iters=20, reps=5):
    """µs per call of ``fn(i)`` (i = call index) from hipGraph replays."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / iters)
    return best


def row(name, us, nbytes=None, flops=None):
    tbs = f"{nbytes / us / 1e6:.2f}" if nbytes else ""
    tf = f"{flops / us / 1e6:.1f}" if flops else ""
    ROWS.append((name, f"{us:.2f}", tbs, tf))
    print(f"{name:58s} {us:9.2f} us  {tbs:>6s} TB/s {tf:>7s} TF/s", flush=True)


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def bench_gemm(M):
    hid, ffn, hq, hkv, d, vocab = 4096, 14336, 32, 8, 128, 128256
    x = bf(M, hid)
    res = bf(M, hid)
    g_in = bf(M, ffn)
    nb = 64
    kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
    cs = ref.rope_cos_sin(8192, d, 500000.0, DEV)
    pos = torch.arange(M, device=DEV, dtype=torch.int64) + 100
    slots = torch.arange(M, device=DEV, dtype=torch.int64) + 40
    shapes = [
        ("qkv  (norm+rope+cache)", (hq + 2 * hkv) * d, hid),
        ("qkv balanced (norm+rope+cache, split remainder)", (hq + 2 * hkv) * d, hid),
        ("o    (+resid)", hid, hq * d),
        ("gate_up (norm+swiglu)", 2 * ffn, hid),
        ("gate_up balanced (norm+swiglu, split remainder)", 2 * ffn, hid),
        ("down (+resid)", hid, ffn),
        ("o    (+resid, split ws as the engine)", hid, hq * d),
        ("down (+resid, split ws as the engine)", hid, ffn),
        ("lm_head (norm)", vocab, hid),
        ("gate_up-plain (norm, unpaired)", 2 * ffn, hid),
    ]
    for name, N, K in shapes:
        nbytes = N * K * 2
        copies = max(2, math.ceil(2**30 / nbytes))
        Ws = [ops.shuffle_weight(bf(N, K, scale=0.02), swiglu=name.startswith("gate_up")) for _ in range(copies)]
        # (the launcher reads RT_SKINNY_CFG once: compare variants from separate processes)
        if name.startswith("qkv balanced"):
            sws = ops.split_workspace(DEV)
            fn = lambda i, sws=sws: ops.skinny_gemm_rope(x, Ws[i % copies], ops.PRO_NORM, pos, cs, kc, vc, slots, hq,
                                                         hkv, d, split_ws=sws)
        elif name.startswith("qkv"):
            fn = lambda i: ops.skinny_gemm_rope(x, Ws[i % copies], ops.PRO_NORM, pos, cs, kc, vc, slots, hq, hkv, d)
        elif "split ws" in name:      # the engine's row-parallel call (parallel/tp.py row_parallel)
            inp = x if name.startswith("o ") else g_in
            sws = ops.split_workspace(DEV)
            fn = lambda i, inp=inp, sws=sws: ops.skinny_gemm(inp, Ws[i % copies], ops.PRO_PLAIN, ops.EPI_RESID, res=res,
                                                             split_ws=sws, split_mode=ops.SPLIT_K)
        elif name.startswith("o ") or name.startswith("down"):
            inp = x if name.startswith("o ") else g_in
            fn = lambda i, inp=inp: ops.skinny_gemm(inp, Ws[i % copies], ops.PRO_PLAIN, ops.EPI_RESID, res=res)
        elif name.startswith("gate_up balanced"):
            sws = ops.split_workspace(DEV)
            fn = lambda i, sws=sws: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM, ops.EPI_SWIGLU, split_ws=sws)
        elif name.startswith("gate_up"):
            fn = lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM, ops.EPI_SWIGLU)
        else:
            fn = lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM)
        us = timed(fn)
        row(f"skinny {name} M={M} N={N} K={K} cfg={os.environ.get('RT_SKINNY_CFG', 'auto')}", us, nbytes, 2 * M * N * K)
        del Ws
        torch.cuda.empty_cache()


def bench_gemm_tp(M, tp, model="llama3-8b"):
    """The per-rank decode GEMMs of a tensor-parallel knight, exactly as forward_decode_fused_tp
    issues them (NORM prologues; o / down with the residual add the all-reduce epilogue carries):
    qkv [(Hq+2Hkv)/tp * D, H], o [H, Hq*D/tp], gate_up [2 F/tp, H], down [H, F/tp], lm_head
    [V/tp, H]. RT_SPLITK / RT_SPLITK_TARGET pin the split (read once per process)."""
    from theroundtaible_amd.models.config import get_config
    c = get_config(model)
    hid, d = c.hidden, c.head_dim
    hq, hkv, ffn = c.n_heads // tp, c.n_kv_heads // tp, c.ffn // tp
    vs = -(-c.vocab // tp)
    vs = -(-vs // 16) * 16
    x, x2, xo = bf(M, hid), bf(M, hid), bf(M, hid)
    a_in, g_in = bf(M, c.n_heads * d // tp), bf(M, ffn)
    nb = 64
    kc = torch.zeros(nb, hkv, 32, d, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nb, hkv, d, 32, dtype=torch.bfloat16, device=DEV)
    cs = ref.rope_cos_sin(8192, d, c.rope_theta, DEV)
    pos = torch.arange(M, device=DEV, dtype=torch.int64) + 100
    slots = torch.arange(M, device=DEV, dtype=torch.int64) + 40
    sw = ops.split_workspace(DEV)
    sk = dict(split_ws=sw, split_mode=ops.SPLIT_K)
    shapes = [("qkv (norm+rope+cache)", (hq + 2 * hkv) * d, hid), ("o (+resid)", hid, hq * d),
              ("gate_up (norm+swiglu)", 2 * ffn, hid), ("down (+resid)", hid, ffn), ("lm_head (norm)", vs, hid)]
    total = 0.0
    for name, N, K in shapes:
        nbytes = N * K * 2
        copies = max(2, math.ceil(2**30 / nbytes))
        rope = name.startswith("qkv")
        Ws = [ops.shuffle_weight(bf(N, K, scale=0.02), swiglu=name.startswith("gate_up"),
                                 rope_heads=hq + hkv if rope else 0, head_dim=d if rope else 0) for _ in range(copies)]
        if rope:   # the decode path never splits qkv (models/llama.py forward_decode_fused_tp)
            fn = lambda i: ops.skinny_gemm_rope(x, Ws[i % copies], ops.PRO_NORM, pos, cs, kc, vc, slots, hq, hkv, d,
                                                split_ws=sw, split_mode=0)
        elif name.startswith("gate_up"):
            fn = lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM, ops.EPI_SWIGLU, **sk)
        elif name.startswith("lm_head"):
            fn = lambda i: ops.skinny_gemm(x, Ws[i % copies], ops.PRO_NORM, ops.EPI_STORE, **sk)
        else:      # row-parallel: the residual add of the all-reduce epilogue, communication elided
            inp = a_in if name.startswith("o ") else g_in
            fn = lambda i, inp=inp: ops.skinny_gemm(inp, Ws[i % copies], ops.PRO_PLAIN, ops.EPI_RESID, res=xo, **sk)
        us = timed(fn)
        T = N // 16 // (2 if name.startswith("gate_up") else 1)
        S = ops.native().splitk_parts(T, K // 32, torch.cuda.get_device_properties(0).multi_processor_count,
                                      ops.SPLIT_WS_INTS)
        total += us * (1 if name.startswith("lm_head") else c.n_layers)
        row(f"tp{tp} {name} M={M} N={N} K={K} tiles={T} splitk={S or 1}", us, nbytes, 2 * M * N * K)
        del Ws
        torch.cuda.empty_cache()
    print(f"tp{tp} {model}: decode GEMMs per step (L x layer + lm_head) = {total:.1f} us", flush=True)
    ROWS.append((f"tp{tp} {model} GEMMs per decode step", f"{total:.1f}", "", ""))


def bench_attn(B, ctx, splits_list):
    hq, hkv, d = 32, 8, 128
    nblk = (ctx + 31) // 32
    copies = 8
    caches = []
    for _ in range(copies):
        kc = bf(B * nblk, hkv, 32, d)
        vc = bf(B * nblk, hkv, d, 32)
        caches.append((kc, vc))
    bt = torch.arange(B * nblk, device=DEV, dtype=torch.int32).reshape(B, nblk)
    cl = torch.full((B,), ctx, device=DEV, dtype=torch.int32)
    q = bf(B, hq, d)
    nbytes = B * ctx * hkv * d * 2 * 2
    for splits in splits_list:
        ws = ops.DecodeWorkspace(B, hq, d, splits, DEV)
        out = torch.empty_like(q)
        # the per-step work plan (as a decode step computes it once for all layers)
        pl = ops.attn_plan(bt, cl, splits, ws, hq, hkv, None, B)
        fn = lambda i, ws=ws, splits=splits, out=out, pl=pl: ops.paged_attention_decode(
            q, caches[i % copies][0], caches[i % copies][1], bt, cl, 1 / math.sqrt(d), splits, ws, out, planned=pl)
        row(f"decode attn B={B} ctx={ctx} splits={splits}", timed(fn), nbytes)


def bench_attn_grouped(B, shared, private, splits_list, hq=32, hkv=8):
    """Shared-prefix groups: B knights read one `shared`-token prefix + `private` own tokens.
    ``hq``/``hkv``: per-rank heads (tensor-parallel shards: 32/tp, 8/tp)."""
    d = 128
    G = hq // hkv
    nsh, npr = shared // 32, (private + 31) // 32
    nblk = nsh + B * npr
    copies = 6
    caches = [(bf(nblk, hkv, 32, d), bf(nblk, hkv, d, 32)) for _ in range(copies)]
    bt = torch.zeros(B, nsh + npr, dtype=torch.int32)
    for b in range(B):
        bt[b, :nsh] = torch.arange(nsh)
        bt[b, nsh:] = nsh + b * npr + torch.arange(npr)
    bt = bt.to(DEV)
    cl = torch.full((B,), nsh * 32 + private, device=DEV, dtype=torch.int32)
    q = bf(B, hq, d)
    groups, _ = ops.decode_groups(["g"] * B, [nsh] * B, G)
    groups = groups.to(DEV)
    nbytes = (nsh * 32 + B * private) * hkv * d * 2 * 2
    for splits in splits_list:
        for grouped in (True, False):
            ws = ops.DecodeWorkspace(B, hq, d, splits, DEV, max_group=16 // G if grouped else 1)
            out = torch.empty_like(q)
            gt = groups if grouped else None
            pl = ops.attn_plan(bt, cl, splits, ws, hq, hkv, gt, B)
            fn = lambda i, ws=ws, splits=splits, out=out, gt=gt, pl=pl: ops.paged_attention_decode(
                q, caches[i % copies][0], caches[i % copies][1], bt, cl, 1 / math.sqrt(d), splits, ws, out, groups=gt,
                planned=pl)
            row(f"decode attn {'grouped' if grouped else 'private'} hq={hq} hkv={hkv} B={B} shared={shared} "
                f"own={private} splits={splits}",
                timed(fn), nbytes if grouped else nbytes + (B - 1) * nsh * 32 * hkv * d * 4)


def bench_sample(B):
    V = 128256
    lg = bf(B, V)
    t = torch.full((B,), 0.8, device=DEV)
    tp = torch.full((B,), 0.9, device=DEV)
    tk = torch.zeros(B, dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.int64)
    offs = torch.zeros(B, device=DEV, dtype=torch.int64)
    out = torch.empty(B, dtype=torch.int64, device=DEV)
    ws = ops.sample_workspace(B, DEV)
    row(f"sample top-p B={B} V={V}", timed(lambda i: ops.sample(lg, t, tp, tk, seeds, offs, out, ws=ws)), B * V * 2)
    tg = torch.zeros(B, device=DEV)
    row(f"sample greedy B={B} V={V}", timed(lambda i: ops.sample(lg, tg, tp, tk, seeds, offs, out, ws=ws)), B * V * 2)
    tk40 = torch.full((B,), 40, dtype=torch.int32, device=DEV)
    row(f"sample top-k 40 (slow path) B={B} V={V}", timed(lambda i: ops.sample(lg, t, tp, tk40, seeds, offs, out, ws=ws)),
        B * V * 2)


def bench_prefill(T, prefix=0):
    """Causal prefill of T new tokens after ``prefix`` cached ones (one sequence, Llama-3-8B heads)."""
    hq, hkv, d = 32, 8, 128
    nblk = (prefix + T + 31) // 32
    kc = bf(nblk, hkv, 32, d)
    vc = bf(nblk, hkv, d, 32)
    q = bf(T, hq, d)
    bt = torch.arange(nblk, device=DEV, dtype=torch.int32)[None]
    cu = torch.tensor([0, T], device=DEV, dtype=torch.int32)
    sp = torch.full((1,), prefix, device=DEV, dtype=torch.int32)
    rows = ops.native().prefill_rows_per_tile(hq // hkv, d)
    tm = ops.prefill_tile_map(cu.cpu(), rows, sp.cpu()).to(DEV)
    flops = 4 * hq * d * T * (prefix + T / 2)
    us = timed(lambda i: ops.prefill_attention(q, kc, vc, bt, cu, sp, 1 / math.sqrt(d), tm), iters=5, reps=3)
    row(f"prefill attn causal T={T} prefix={prefix}", us, None, flops)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=3)
    ap.add_argument("--ctx", type=int, default=6000)
    ap.add_argument("--only", default="gemm,attn,sample,prefill")
    ap.add_argument("--splits", default="4,8,11,16,32")
    ap.add_argument("--shared", default="22000:1500", help="grouped attention: shared:private tokens list, comma-sep")
    ap.add_argument("--tp", default="2,4,8", help="gemm_tp: tensor-parallel degrees of the shard shapes")
    ap.add_argument("--model", default="llama3-8b", help="gemm_tp: model preset")
    ap.add_argument("--prefill", default="4096:0", help="prefill: new:prefix token counts, comma-sep")
    a = ap.parse_args()
    only = set(a.only.split(","))
    torch.manual_seed(0)
    if "gemm" in only:
        bench_gemm(a.batch)
    if "gemm_tp" in only:
        for tp in (int(t) for t in a.tp.split(",")):
            bench_gemm_tp(a.batch, tp, a.model)
    if "attn" in only:
        bench_attn(a.batch, a.ctx, [int(s) for s in a.splits.split(",")])
        bench_attn(a.batch, 1500, [4, 8, 11, 16])
    if "gattn" in only:
        for tp in (int(t) for t in a.tp.split(",")):
            for sp in a.shared.split(","):
                sh, pr = (int(x) for x in sp.split(":"))
                bench_attn_grouped(a.batch, sh, pr, [int(s) for s in a.splits.split(",")], 32 // tp, max(1, 8 // tp))
    if "sample" in only:
        bench_sample(a.batch)
    if "prefill" in only:
        for pf in a.prefill.split(","):
            t, pre = (int(x) for x in pf.split(":"))
            bench_prefill(t, pre)
    print("\n| op | us | TB/s | TF/s |\n|---|---|---|---|")
    for r in ROWS:
        print("| " + " | ".join(r) + " |")


if __name__ == "__main__":
    main()
