"""Probe: is ONE persistent launch per layer (tools/experiments/decode_layer.hip) faster than the
six-launch fused decode layer at the tensor-parallel tp8 SHARD shapes of Llama-3-8B?

VERDICT r3 "do this" #1 asks whether folding the layer into fewer launches pays once the GEMMs
are ramp-bound (tp 8: hidden 4096, 4 query heads / 1 KV head per rank, FFN shard 1792). Both
paths run the same shard-shaped model (collectives elided, as in ``bench.py --simulate-tp``),
3 private sequences of CTX tokens, captured as hipGraphs of L layers, timed over replays.
The persistent kernel has no split-K (qkv 48 tiles, gate_up 112 tiles on 48 / 112 CUs) — the
comparison is of whole layers as they are. Needs ``python tools/experiments/build_exp.py``.

    python tools/probes/persistent_tp8.py [--ctx 8192] [--layers 8] [--splits 16,32,64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "experiments"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.engine import Engine, EngineConfig  # noqa: E402
from theroundtaible_amd.models import config as mcfg  # noqa: E402
from theroundtaible_amd.models.llama import AttnMeta  # noqa: E402

DEV = "cuda"


def timed(fn, reps=20):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=8192)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--splits", default="16,32,64")
    a = ap.parse_args()
    mcfg.PRESETS["tp8shard"] = mcfg.ModelConfig("tp8shard", "llama", a.layers, 4096, 4, 1, 128, 1792, 32000,
                                                131072, 500000.0, 1e-5)
    from build_exp import load
    exp = load()
    nb = 3 * (a.ctx // 32 + 4) + 64
    e = Engine(EngineConfig(model="tp8shard", weights="random-full:5", device=DEV, num_blocks=nb, use_graphs=False))
    m, kv = e.model, e.kv
    m.force_tp_path = True
    g = torch.Generator().manual_seed(3)
    seqs = [kv.seq(f"s{i}") for i in range(3)]
    for s in seqs:
        ids = torch.randint(0, 32000, (a.ctx,), generator=g).tolist()
        e.prefill([(s, ids)])
    for s in seqs:
        kv.ensure_capacity(s, s.length + 1)
    pos = torch.tensor([s.length for s in seqs], device=DEV)
    slots = torch.tensor([s.blocks[p // 32] * 32 + p % 32 for s, p in zip(seqs, pos.tolist())], device=DEV)
    maxb = max(len(s.blocks) for s in seqs)
    bt = torch.zeros(3, maxb, dtype=torch.int32)
    for j, s in enumerate(seqs):
        bt[j, :len(s.blocks)] = torch.tensor(s.blocks)
    bt = bt.to(DEV)
    ctx = (pos + 1).to(torch.int32)
    tok = torch.tensor([5, 7, 11], device=DEV)
    dec = m.decode_weights()
    out = {"ctx": a.ctx, "layers": a.layers, "rows": []}
    for S in [int(x) for x in a.splits.split(",")]:
        ws = ops.DecodeWorkspace(3, m.n_heads, m.head_dim, S, DEV)
        meta = AttnMeta("decode", slots, bt, ctx, num_splits=S, workspace=ws)
        res0 = F.embedding(tok, m.w["embed"]).contiguous()
        res = res0.clone()

        def six():
            res.copy_(res0)
            m.forward(tok, pos, kv, meta, hidden=res)

        M, D = 3, m.head_dim
        q = torch.empty(M, m.n_heads, D, dtype=res.dtype, device=DEV)
        att = torch.empty(M, m.n_heads * D, dtype=res.dtype, device=DEV)
        gg = torch.empty(M, dec["layers"][0]["w_down"].shape[1], dtype=res.dtype, device=DEV)

        def pers():
            res.copy_(res0)
            for l, lw in enumerate(dec["layers"]):
                exp.decode_layer(res, q, att, gg, lw["wqkv"], lw["wo"], lw["w_gate_up"], lw["w_down"], pos, m.cos_sin,
                                 kv.k_layer(l), kv.v_layer(l), slots, bt, ctx, ws.partial_o, ws.partial_ml,
                                 ws.counters, ws.sync, ws.err, m.n_heads, m.n_kv_heads, S, m.cfg.norm_eps, m.scale)
            ops.skinny_gemm(res, dec["lm_head"], ops.PRO_NORM, ops.EPI_STORE, eps=m.cfg.norm_eps)

        t6 = timed(six)
        tp = timed(pers)
        err = int(ws.err.item())
        row = {"splits": S, "six_launch_us_per_step": round(t6, 1), "persistent_us_per_step": round(tp, 1),
               "six_per_layer_us": round(t6 / a.layers, 2), "persistent_per_layer_us": round(tp / a.layers, 2),
               "persistent_poll_expired": err}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
