#!/usr/bin/env python3
"""Tensor-parallel numerics check on the GPU: a tp=N engine against a tp=1 engine with the SAME
weights (``random-dev:<seed>``: full tensors generated on the device, then sharded).

One process per rank (torchrun). Ranks may share one GPU (ROUNDTABLE_DIST_BACKEND=gloo, the
1-GPU rehearsal: K9 between the ranks' IPC buffers, host-staged RCCL-free prefill all-reduce)
or own one each (RCCL + K9 over xGMI). Every rank:

1. prefills a fixed prompt (column/row-parallel hipBLASLt GEMMs + C2 all-reduce) -> logits;
2. runs ONE fused decode step by hand (shard GEMMs, K9 one-shot all-reduces adding into the
   residual, vocab-parallel lm_head + C3 all-gather) -> logits;
3. greedy-decodes ``--tokens`` tokens through ``run_turns`` (C3 distributed argmax; with
   ``--graphs`` the captured decode step, replayed once per token on every rank).

Rank 0 writes {prefill_logits, decode_logits, ids, ...} to ``--out`` (torch.save). The tp=1
reference is the same script with ``--nproc-per-node 1``; tests/test_distributed_gpu.py compares.

    torchrun --nproc-per-node 4 tools/tp_check.py --model llama3-70b --layers 2 --out /tmp/tp4.pt
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--tokens", type=int, default=12)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--graphs", action="store_true",
                    help="hipGraph decode: RCCL groups, or gloo groups whose every in-step collective is K9")
    ap.add_argument("--poll-limit", type=int, default=0,
                    help="K9 flag-wait bound in polls (0 = the comm's default): a rehearsal whose ranks share a "
                         "GPU fails fast instead of spinning if the scheduler does not co-run their grids")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    from theroundtaible_amd.models.llama import AttnMeta
    from theroundtaible_amd.parallel.cluster import init_cluster, shutdown_cluster
    from theroundtaible_amd.parallel.tp import TPInfo

    cl = init_cluster(prefer_gpu=True)
    tp = None
    if cl.world > 1:
        import torch.distributed as dist
        tp = TPInfo(size=cl.world, rank=cl.rank, group=dist.group.WORLD)
    e = Engine(EngineConfig(model=a.model, weights=f"random-dev:{a.seed}", device=cl.device, dtype="bf16",
                            max_kv_tokens=4096, kv_cache_fraction=0.05, use_graphs=a.graphs,
                            weight_residency="dual", model_overrides={"n_layers": a.layers}), tp)
    if a.poll_limit and getattr(e.tp, "oneshot", None) is not None:
        e.tp.oneshot.set_poll_limit(a.poll_limit)
    prompt = "De ronde tafel bespreekt tensor-parallelle ridders over xGMI. " * 6
    ids = e.encode_prompt(prompt)
    s = e.kv.seq("probe")
    pre = e.prefill([(s, ids)]).float()                     # [1, V]
    # one fused decode step by hand (the path a captured step runs)
    e.kv.ensure_capacity(s, s.length + 1)
    dev = e.device
    p = s.length
    pos = torch.tensor([p], device=dev)
    slots = torch.tensor([s.blocks[p // e.kv.block_size] * e.kv.block_size + p % e.kv.block_size], device=dev)
    bt = torch.zeros(1, len(s.blocks), dtype=torch.int32)
    bt[0] = torch.tensor(s.blocks, dtype=torch.int32)
    meta = AttnMeta("decode", slots, bt.to(dev), (pos + 1).to(torch.int32), num_splits=4)
    fused = e.model.fused_decode_ok(torch.tensor([1], device=dev))
    dec = e.model.forward(torch.tensor([int(pre.argmax())], device=dev), pos, e.kv, meta).float()
    e.release("probe")
    sp = SamplingParams(temperature=0.0, max_new_tokens=a.tokens, ignore_eos=True, stop_on_consensus=False)
    outs = e.run_turns([Turn("K1", prompt, sp), Turn("K2", prompt + " Tweede ridder.", sp)])
    flag_errors = e.device_flag_errors()
    per_rank = cl.all_gather_object({"replays": int(e.stats.get("graph_replays", 0)),
                                     "graphs": bool(e.ecfg.use_graphs),
                                     "fallbacks": int(e.stats.get("capture_fallbacks", 0)),
                                     "fused_ar_calls": int(getattr(e.tp, "fused_ar_calls", 0))})
    rec = {"world": cl.world, "backend": cl.backend, "fused": bool(fused),
           "graph_replays_per_rank": [r["replays"] for r in per_rank],
           "graphs_per_rank": [r["graphs"] for r in per_rank],
           "capture_fallbacks": sum(r["fallbacks"] for r in per_rank),
           "fused_ar_calls_per_rank": [r["fused_ar_calls"] for r in per_rank],
           "k9": bool(getattr(e.tp, "oneshot", None)),
           "fused_ar": bool(getattr(getattr(e.tp, "oneshot", None), "fused", False)),
           "fused_ar_calls": int(getattr(e.tp, "fused_ar_calls", 0)), "prefill_logits": pre[0].cpu(), "decode_logits": dec[0].cpu(),
           "ids": [o.ids for o in outs], "errors": [str(o.error) if o.error else None for o in outs],
           "flag_errors": flag_errors}
    if cl.rank == 0:
        torch.save(rec, a.out)
        print(f"tp_check world={cl.world} fused={fused} k9={rec['k9']} fused_ar={rec['fused_ar_calls']} ids={rec['ids']}", flush=True)
    cl.barrier()
    shutdown_cluster()
    return 0


if __name__ == "__main__":
    sys.exit(main())
