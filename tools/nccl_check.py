#!/usr/bin/env python3
"""RCCL data-plane check on real hardware, one process per GPU (torchrun, any world size >= 1).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/nccl_check.py

A 1-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so the
multi-rank tests rehearse over gloo; this script runs the exact RCCL calls of the scaling
bench and the TP decode path with ``backend="nccl"`` at whatever world size it is given —
world 1 on a 1-GPU box, 8 on a node:

* ``init_process_group(backend="nccl", device_id=cuda:LOCAL_RANK)`` (eager communicator) plus
  the gloo control group, via ``parallel/cluster.py::init_cluster``;
* C1: ``TokenExchange`` (static-shape async all-gather of token ids on the device) and the
  shape-agreeing ``exchange_token_ids`` fallback;
* ``barrier(device_ids=...)``;
* C2/C3 under hipGraph capture: ``dist.all_reduce`` of a decode-size bf16 vector and
  ``dist.all_gather`` of (value, id) pairs captured into one graph, replayed, checked;
* ``TPInfo.all_reduce`` / ``greedy_gather`` / ``all_gather_last`` on an RCCL group.

Rank 0 prints ONE JSON line ``{"ok": true, "world": N, "backend": "nccl", "checks": k}``.
"""
from __future__ import annotations

import json
import os
import sys

os.environ.setdefault("ROUNDTABLE_DIST_BACKEND", "nccl")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from theroundtaible_amd.parallel.cluster import init_cluster, shutdown_cluster  # noqa: E402
from theroundtaible_amd.parallel.exchange import TokenExchange, exchange_token_ids  # noqa: E402
from theroundtaible_amd.parallel.tp import TPInfo  # noqa: E402


def main() -> int:
    cl = init_cluster(prefer_gpu=True, timeout_s=300)
    assert cl.backend == "nccl" and dist.is_initialized() and dist.get_backend() == "nccl", cl
    dev = torch.device(cl.device)
    W, r = cl.world, cl.rank
    checks = 0

    # C1, static shapes: every rank leads two knights (slots 2r, 2r+1)
    ex = TokenExchange(cl, rows=2, width=32, device=cl.device)
    mine = [(2 * r, [r, 1, 2, 3]), (2 * r + 1, list(range(r + 5)))]
    ex.start(mine)
    got = ex.wait()
    want = {}
    for k in range(W):
        want[2 * k] = [k, 1, 2, 3]
        want[2 * k + 1] = list(range(k + 5))
    assert got == want, (got, want)
    checks += 1
    # C1 fallback (shape agreement over gloo, data over RCCL)
    got = exchange_token_ids(cl, [(100 + r, [r] * (3 + r))], cl.device)
    assert got == {100 + k: [k] * (3 + k) for k in range(W)}, got
    checks += 1
    cl.barrier()
    checks += 1

    # C2 / C3 captured in one hipGraph, as the TP decode step does
    world_group = dist.group.WORLD
    x = torch.empty(4096, dtype=torch.bfloat16, device=dev)
    pair = torch.empty(3, 2, dtype=torch.float32, device=dev)
    parts = [torch.empty_like(pair) for _ in range(W)]

    def body():
        dist.all_reduce(x, group=world_group)
        dist.all_gather(parts, pair, group=world_group)

    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        x.fill_(1.0)
        pair.fill_(float(r))
        body()                               # warm-up outside capture
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for rep in range(3):
        x.fill_(float(r + 1 + rep))
        pair.fill_(float(10 * r + rep))
        g.replay()
        torch.cuda.synchronize(dev)
        exp = sum(float(k + 1 + rep) for k in range(W))
        assert torch.allclose(x.float(), torch.full_like(x.float(), exp)), (x[:4], exp)
        for k in range(W):
            assert torch.equal(parts[k], torch.full_like(pair, float(10 * k + rep))), (k, parts[k])
        checks += 1

    # TPInfo on an RCCL group (size W; at W = 1 its collectives are identities by design)
    tp = TPInfo(size=W, rank=r, group=world_group)
    y = torch.full((16,), float(r + 1), dtype=torch.bfloat16, device=dev)
    tp.all_reduce(y)
    assert float(y[0]) == float(sum(k + 1 for k in range(W)))
    logits = torch.randn(3, 64, device=dev)
    logits[:, 5 + r] += 100.0 + r           # rank W-1 holds the global max
    ids = tp.greedy_gather(logits, vocab=64 * W)
    assert ids.tolist() == [(W - 1) * 64 + 5 + (W - 1)] * 3, ids
    full = tp.all_gather_last(torch.full((2, 8), float(r), device=dev))
    assert full.shape == (2, 8 * W) and float(full[0, -1]) == float(W - 1)
    checks += 3

    rec = {"ok": True, "world": W, "backend": cl.backend, "device": cl.device, "checks": checks,
           "rccl_version": ".".join(map(str, torch.cuda.nccl.version())) if hasattr(torch.cuda, "nccl") else None}
    recs = cl.all_gather_object(rec)
    if r == 0:
        out = dict(recs[0])
        out["ranks_ok"] = sum(1 for x in recs if x.get("ok"))
        os.write(1, (json.dumps(out) + "\n").encode())
    cl.barrier()
    shutdown_cluster()
    return 0


if __name__ == "__main__":
    sys.exit(main())
