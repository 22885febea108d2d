"""First-contact failure containment and the multi-rank agreement rounds, on
CPU gloo ranks: a stage that raises or stalls on ONE rank ends the whole bench with one JSON
line from rank 0 naming the stage, rc != 0, inside the stage timeout; the graph-capture fallback
is decided by the whole TP group; serve --tp ranks agree on one KV pool and on every outcome."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_distributed_cpu import ROOT, free_port


def _bench_fault(nproc, fault, extra=(), timeout=240):
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--device", "cpu", "--model", "tiny-llama", "--steps", "2", "--warmup", "1",
           "--new-tokens", "6", "--temperature", "0", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1", ROUNDTABLE_BENCH_FAULT=fault)
    t0 = time.monotonic()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, lines, time.monotonic() - t0


def test_bench_rank_failure_at_load_reports_stage():
    """Rank 1 raises while loading its engine: rank 0 prints ONE JSON line naming the stage and
    rank, and the launch exits non-zero (no hang in rank 0's next collective)."""
    r, lines, _ = _bench_fault(2, "1:engine_load:raise")
    assert r.returncode != 0
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(lines[0])
    assert out["value"] is None and out["n_gpus"] == 2
    assert out["failed_stage"] == "engine_load" and out["failed_rank"] == 1
    assert "injected failure" in out["error"]


def test_bench_collective_stall_on_one_rank_ends_within_timeout():
    """Rank 1 stalls when round 2 starts (its peers wait in the round's collectives): every rank's
    stage limit expires, rank 0 reports the stalled stage and the run ends well inside the
    launcher's patience — never the 1800-s process-group default."""
    r, lines, took = _bench_fault(2, "1:round 2:stall", ("--stage-timeout", "8"))
    assert r.returncode != 0
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(lines[0])
    assert out["failed_stage"] == "round 2" and "stalled" in out["error"]
    assert {f["failed_rank"] for f in out["failures"]} <= {0, 1}
    assert took < 120, took


def test_bench_raise_on_rank_zero_mid_run():
    r, lines, _ = _bench_fault(2, "0:round 3:raise")
    assert r.returncode != 0 and len(lines) == 1
    out = json.loads(lines[0])
    assert out["failed_stage"] == "round 3" and out["failed_rank"] == 0


def _capture_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.engine.engine import Engine
        from theroundtaible_amd.engine import EngineConfig
        from theroundtaible_amd.parallel.tp import TPInfo
        # the agreement logic alone: an engine shell whose capture fails on rank 1 only
        e = object.__new__(Engine)
        e.on_gpu = True
        e.ecfg = EngineConfig(device="cpu")
        e.tp = TPInfo(size=world, rank=rank, group=dist.group.WORLD)
        e.graphs = {"stale": object()}
        e.stats = {}

        def graph_for(B, max_ctx, grouped=False, dist_greedy=False):
            if rank == 1:
                raise RuntimeError("operation not permitted when stream is capturing")
            return "graph"

        e._graph_for = graph_for
        got = e._agreed_graph(3, 100, True, False)
        q.put((rank, got, e.ecfg.use_graphs, len(e.graphs), e.stats.get("capture_fallbacks")))
    finally:
        dist.destroy_process_group()


def test_capture_fallback_is_agreed_by_the_group():
    """A capture that fails on ONE rank of a TP group sends every rank to eager decode (the ranks
    that captured drop their graphs): no rank replays K9 calls its peers never issue."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_capture_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        got, use_graphs, n_graphs, fallbacks = res[rank]
        assert got is None and use_graphs is False and n_graphs == 0 and fallbacks == 1, (rank, res[rank])


def _pool_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.engine import Engine, EngineConfig
        from theroundtaible_amd.parallel.tp import TPInfo
        tp = TPInfo(size=world, rank=rank, group=dist.group.WORLD)
        # unequal per-rank budgets (what two rehearsal ranks on one GPU see from mem_get_info)
        per_block = 2 * 2 * 1 * 64 * 32 * 4 * 2
        e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", weights="random-full:3",
                                kv_budget_bytes=(96 if rank == 0 else 160) * per_block), tp)
        q.put((rank, e.kv.num_blocks))
    finally:
        dist.destroy_process_group()


def test_tp_ranks_agree_on_one_kv_pool():
    """every rank of a TP engine holds the same number of KV blocks (the group
    minimum), so the allocators decide identically and KVCacheOOM hits all ranks or none."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_pool_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]


def _mirror_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from theroundtaible_amd.parallel.cluster import init_cluster, shutdown_cluster
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank))
    cl = init_cluster(prefer_gpu=False, timeout_s=60)
    try:
        from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
        from theroundtaible_amd.parallel.tp import TPInfo
        from theroundtaible_amd.serve import MirroredEngine, serve_follower
        tp = TPInfo(size=world, rank=rank, group=dist.group.WORLD)
        e = Engine(EngineConfig(model="tiny-llama", device="cpu", dtype="fp32", weights="random-full:3",
                                num_blocks=128), tp)
        if rank == 1:   # the follower's engine fails its 2nd call (an outcome rank 0 does not share)
            calls, real = [0], e.start_turns

            def flaky(turns):
                calls[0] += 1
                out = real(turns)       # the collectives ran on every rank; the host step after fails
                if calls[0] == 2:
                    raise ValueError("follower-only failure")
                return out

            e.start_turns = flaky
        p = SamplingParams(temperature=0, max_new_tokens=4, ignore_eos=True, stop_on_consensus=False)
        if rank == 0:
            m = MirroredEngine(e, cl)
            first = m.start_turns([Turn("a", "eerste ridder", p)])
            errs = []
            for key in ("b", "c"):
                try:
                    m.start_turns([Turn(key, "tweede ridder", p)])
                except RuntimeError as ex:
                    errs.append(str(ex))
            m.stop_followers()
            q.put((rank, len(first), errs, m.diverged is not None))
        else:
            q.put((rank, serve_follower(e, cl), [], None))
    finally:
        shutdown_cluster()


def test_serve_tp_outcome_mismatch_stops_the_group():
    """followers report every operation's outcome; when a follower's differs
    from rank 0's (here an error on the follower only) the group stops — the follower leaves
    its loop, rank 0 refuses later operations instead of entering collectives nobody joins."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_mirror_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=180) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_first, errs, diverged = res[0]
    assert n_first == 1 and diverged is True
    assert len(errs) == 2 and "disagree" in errs[0] and "stopped" in errs[1]
    assert res[1][0] == 2          # the follower ran 2 operations, then left


@pytest.mark.parametrize("nproc,tp", [(8, 4), (4, 2)])
def test_config5_topology_two_tp_groups(nproc, tp):
    """BASELINE config 5 on gloo ranks: two disjoint TP groups, one knight each.
    C1 crosses the groups from the group leaders only, no turn fails, and the greedy transcript
    equals the same two-knight table on ONE rank."""
    from test_distributed_cpu import _bench, _bench_single
    common = ("--knights-per-table", "2", "--weights", "random-full:5")
    two = _bench(nproc, ("--tp", str(tp), "--knights-per-gpu", "1", *common))
    one = _bench_single(("--temperature", "0", *common))
    d = two["detail"]
    assert two["config"]["knights"] == 2 and two["config"]["tp"] == tp
    assert d["failed_turns"] == 0 and one["detail"]["failed_turns"] == 0
    lead = [0, tp]
    contrib = d["c1_contributions_per_rank"]
    assert all((c > 0) == (r in lead) for r, c in enumerate(contrib)), contrib
    assert d["decode_tokens"] == one["detail"]["decode_tokens"]
    assert d["transcript_sha"] == one["detail"]["transcript_sha"]
