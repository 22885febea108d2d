"""Probe (VERDICT r4 next #1b): does a two-micro-batch, two-stream captured decode step hide the
tensor-parallel all-reduces of a tp >= 4 shard under the other micro-batch's compute?

Both schedules run the Llama-3-8B rank-0 SHARD shapes of a tp = N knight (hidden 4096, 32/N query
heads, 8/N KV heads, FFN 14336/N; N = 8: 4 / 1 / 1792), 3 private sequences of CTX tokens, L
layers + the vocab-sharded lm_head, captured as one hipGraph and timed over replays. Every
all-reduce is the device-side stand-in of ``bench.py --simulate-tp`` (parallel/tp.py
SimulatedTP: a kernel holding the K9 launch's CUs for COMM µs, in the graph):

* ``one``: the engine's step — ONE stream, M = 3 rows, per layer qkv -> attention (+ combine)
  -> o + all-reduce -> gate_up -> down + all-reduce;
* ``two``: rows {0, 1} on the capture stream and row {2} on a second stream (fork / join events
  in the graph), each with its own split-K / attention workspaces, the same per-layer chain; the
  lm_head runs once on the joined rows. While one micro-batch waits in its all-reduce the other
  can compute — the overlap the review asked to measure.

    python tools/probes/microbatch_tp8.py [--tp 8] [--ctx 8192] [--layers 8] [--comm 0,5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from theroundtaible_amd import ops  # noqa: E402
from theroundtaible_amd.engine import Engine, EngineConfig  # noqa: E402
from theroundtaible_amd.models import config as mcfg  # noqa: E402
from theroundtaible_amd.parallel.tp import SimulatedTP  # noqa: E402

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
    best = float("inf")
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


class Micro:
    """One micro-batch's rows, metadata views and private workspaces."""

    def __init__(self, m, r0, r1, slots, bt, ctx, pos, splits):
        self.r0, self.r1 = r0, r1
        self.slots, self.bt, self.ctx, self.pos = slots[r0:r1], bt[r0:r1], ctx[r0:r1], pos[r0:r1]
        self.ws = ops.DecodeWorkspace(r1 - r0, m.n_heads, m.head_dim, splits, DEV)
        self.sw = ops.split_workspace(DEV)
        self.splits = splits


def layer_chain(m, kv, tp, res, mb, l, lw, eps):
    from theroundtaible_amd.models.llama import AttnMeta
    B = mb.r1 - mb.r0
    meta = AttnMeta("decode", mb.slots, mb.bt, mb.ctx, num_splits=mb.splits, workspace=mb.ws)
    kc, vc = kv.k_layer(l), kv.v_layer(l)
    q = ops.skinny_gemm_rope(res, lw["wqkv"], ops.PRO_NORM, mb.pos, m.cos_sin, kc, vc, mb.slots, m.n_heads,
                             m.n_kv_heads, m.head_dim, eps, split_ws=mb.sw, split_mode=0)
    a = m.attention(q, kc, vc, meta)
    tp.row_parallel(a.reshape(B, -1), lw["wo"], res=res, split_ws=mb.sw, split_mode=ops.SPLIT_K)
    g = ops.skinny_gemm(res, lw["w_gate_up"], ops.PRO_NORM, ops.EPI_SWIGLU, eps=eps, split_ws=mb.sw,
                        split_mode=ops.SPLIT_K)
    tp.row_parallel(g, lw["w_down"], res=res, split_ws=mb.sw, split_mode=ops.SPLIT_K)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=8192)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--comm", default="0,5", help="µs per simulated all-reduce (list)")
    ap.add_argument("--gather", type=float, default=9.5)
    a = ap.parse_args()
    T = a.tp
    mcfg.PRESETS["shard"] = mcfg.ModelConfig("shard", "llama", a.layers, 4096, 32 // T, max(1, 8 // T), 128,
                                             14336 // T, 128256 // T, 131072, 500000.0, 1e-5)
    nb = 3 * (a.ctx // 32 + 4) + 64
    e = Engine(EngineConfig(model="shard", weights="random:5", device=DEV, num_blocks=nb, use_graphs=False))
    m, kv = e.model, e.kv
    m.force_tp_path = True
    g = torch.Generator().manual_seed(3)
    seqs = [kv.seq(f"s{i}") for i in range(3)]
    for s in seqs:
        ids = torch.randint(0, m.cfg.vocab, (a.ctx,), generator=g).tolist()
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
    eps = m.cfg.norm_eps
    S = ops.decode_splits(3, m.n_kv_heads)
    S1, S2 = ops.decode_splits(2, m.n_kv_heads), ops.decode_splits(1, m.n_kv_heads)
    res0 = F.embedding(tok, m.w["embed"]).contiguous()
    res = res0.clone()
    out = {"tp": T, "ctx": a.ctx, "layers": a.layers, "splits": [S, S1, S2], "rows": []}
    for comm in (float(c) for c in a.comm.split(",")):
        tp = SimulatedTP(T, comm_us=comm or None, gather_us=a.gather if comm else None)
        if comm:
            tp.calibrate_stand_in()
        one_mb = Micro(m, 0, 3, slots, bt, ctx, pos, S)
        mbs = [Micro(m, 0, 2, slots, bt, ctx, pos, S1), Micro(m, 2, 3, slots, bt, ctx, pos, S2)]
        side = torch.cuda.Stream()

        def one():
            res.copy_(res0)
            for l, lw in enumerate(dec["layers"]):
                layer_chain(m, kv, tp, res, one_mb, l, lw, eps)
            tp.all_gather_last(ops.skinny_gemm(res, dec["lm_head"], ops.PRO_NORM, ops.EPI_STORE, eps=eps,
                                               split_ws=one_mb.sw, split_mode=ops.SPLIT_K))

        def two():
            res.copy_(res0)
            r_a, r_b = res[0:2], res[2:3]
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)                       # fork
            for l, lw in enumerate(dec["layers"]):
                layer_chain(m, kv, tp, r_a, mbs[0], l, lw, eps)
                with torch.cuda.stream(side):
                    layer_chain(m, kv, tp, r_b, mbs[1], l, lw, eps)
            cur.wait_stream(side)                       # join
            tp.all_gather_last(ops.skinny_gemm(res, dec["lm_head"], ops.PRO_NORM, ops.EPI_STORE, eps=eps,
                                               split_ws=one_mb.sw, split_mode=ops.SPLIT_K))

        t1 = timed(one)
        r1 = res.clone()
        t2 = timed(two)
        same = bool(torch.equal(r1, res))
        row = {"comm_us": comm, "one_stream_us_per_step": round(t1, 1), "two_stream_us_per_step": round(t2, 1),
               "one_per_layer_us": round(t1 / a.layers, 2), "two_per_layer_us": round(t2 / a.layers, 2),
               "residual_bits_equal": same}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
