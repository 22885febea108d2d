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


class _FakeK9:
    """Stand-in for the K9 comm: a host call counter; resync() is the real agreement shape (group
    MAX over the TP group, then a second all-reduce as the barrier)."""

    def __init__(self, group, calls):
        self.group, self.calls, self.resyncs = group, calls, 0

    def resync(self):
        t = torch.tensor([float(self.calls)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.calls = int(t.item())
        dist.all_reduce(torch.zeros(1, dtype=torch.float64), group=self.group)
        self.resyncs += 1
        return True


def _capture_worker(rank, world, port, q, where):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.engine import graphs
        from theroundtaible_amd.engine.engine import Engine
        from theroundtaible_amd.engine import EngineConfig
        from theroundtaible_amd.parallel.tp import TPInfo

        class CountingTP(TPInfo):
            agreements = 0

            def any_rank(self, flag):
                CountingTP.agreements += 1
                return super().any_rank(flag)

        # the agreement logic alone: an engine shell whose graph set-up fails on rank 1 only,
        # either allocating the graph's buffers or inside the capture (whose eager warm-up runs
        # issue K9 calls: rank 0 has issued 4 of them, rank 1 only 1)
        e = object.__new__(Engine)
        e.on_gpu = True
        e.ecfg = EngineConfig(device="cpu")
        e.tp = CountingTP(size=world, rank=rank, group=dist.group.WORLD)
        e.tp.oneshot = _FakeK9(dist.group.WORLD, 10)
        e.graphs = {(0, 8, False, False): "cached graph"}
        e.stats = {}
        e._graph_key = lambda B, grouped, dist_greedy: (B, 8, grouped, dist_greedy)

        class FakeGraph:
            def __init__(self, engine, bucket, splits, grouped=False, dist_greedy=False, capture=True):
                if where == "alloc" and rank == 1:
                    raise RuntimeError("HIP out of memory allocating the graph's buffers")

            def capture(self):
                e.tp.oneshot.calls += 1 if rank == 1 else 4
                if where == "capture" and rank == 1:
                    raise RuntimeError("operation not permitted when stream is capturing")

        graphs.DecodeGraph = FakeGraph
        cached = e._agreed_graph(0, 100, False, False)
        n_cached = CountingTP.agreements
        got = e._agreed_graph(3, 100, True, False)
        q.put((rank, cached, n_cached, got, e.ecfg.use_graphs, len(e.graphs), e.stats.get("capture_fallbacks"),
               e.tp.oneshot.calls, e.tp.oneshot.resyncs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("where", ["alloc", "capture"])
def test_capture_fallback_is_agreed_by_the_group(where):
    """A graph set-up that fails on ONE rank of a TP group sends every rank to eager decode (the
    ranks that captured drop their graphs): no rank replays K9 calls its peers never issue. A
    failure inside the capture (after the warm-up's K9 calls) also re-agrees the ranks' K9 call
    counters (advisor r4: the counters drifted apart and every later call waited out its bound);
    a buffer failure is agreed before any call is issued. A cached graph costs no agreement."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_capture_worker, args=(r, 2, port, q, where)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        cached, n_cached, got, use_graphs, n_graphs, fallbacks, calls, resyncs = res[rank]
        assert cached == "cached graph" and n_cached == 0, res[rank]
        assert got is None and use_graphs is False and n_graphs == 0 and fallbacks == 1, (rank, res[rank])
        if where == "capture":
            assert resyncs == 1 and calls == 14, res[rank]      # both ranks at the group max
        else:
            assert resyncs == 0 and calls == 10, res[rank]      # no call was issued


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


def test_discuss_tp2_knight_skipped_when_a_rank_stalls(tmp_path):
    """containment outside the bench. A plain ``roundtable discuss`` whose Groot
    knight is tensor-parallel over 2 ranks; rank 1 stalls for 20 s on entering round 1's turn
    (before any collective of it). Every rank of Groot's group takes the SAME decision at the
    turn-start rendezvous (launcher store, knights/distributed.py): the turn is skipped with a
    timeout error after the 6-s turn timeout on rank 0 (the reference skips a failed knight and the
    round goes on, /root/reference/src/orchestrator.ts:521-535), the late rank joins that decision
    instead of entering collectives its peer abandoned, Klein (tp 1) speaks, and round 2 runs
    with both knights."""
    from test_distributed_cpu import _tp_project
    _tp_project(tmp_path, {"Groot": {"tp": 2}, "Klein": {}})
    cfg_path = tmp_path / ".roundtable" / "config.json"
    cfg = json.loads(cfg_path.read_text())
    cfg["rules"].update(max_rounds=2, timeout_per_turn_seconds=6)
    cfg_path.write_text(json.dumps(cfg))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               ROUNDTABLE_BENCH_FAULT="1:turn 1:sleep20")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-m", "theroundtaible_amd", "discuss", "TP onderwerp", "--no-read-codebase",
                        "--choice", "4"], capture_output=True, text=True, timeout=400, env=env, cwd=str(tmp_path))
    took = time.monotonic() - t0
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    sessions = os.listdir(tmp_path / ".roundtable" / "sessions")
    disc = (tmp_path / ".roundtable" / "sessions" / sessions[0] / "discussion.md").read_text()
    assert "Round 1 — Klein" in disc and "Round 1 — Groot" not in disc, disc[:2000]
    assert "Round 2 — Groot" in disc and "Round 2 — Klein" in disc, disc[:2000]
    assert "did not reach the turn within 6 s" in r.stdout + r.stderr, r.stdout[-2000:]
    # timestamped stage transitions name where each rank is
    assert "stage 'turn 1'" in r.stderr and "stage 'turn 2'" in r.stderr
    assert took < 200, took


def test_discuss_tp2_waits_for_a_slow_loading_rank(tmp_path):
    """ranks load their engines one after another, and a real checkpoint can
    take minutes longer on one rank than on its peers. Those peers must wait for it under the LOAD
    limit (the load-timeout gloo groups of parallel/cluster.py: the TP group meets there after
    loading its weights, and every rank meets there after building all its engines), not inside a
    short-timeout collective. Here the containment timeout of every collective is 10 s and rank 0
    enters each load stage 15 s late: its second engine (Klein, tp 1) loads after Groot's TP group
    set-up, while rank 1 has nothing left to load. The run still completes, both knights speak
    (before the load groups, rank 1 died in its first control collective after 10 s)."""
    from test_distributed_cpu import _tp_project
    _tp_project(tmp_path, {"Groot": {"tp": 2}, "Klein": {}})
    cfg_path = tmp_path / ".roundtable" / "config.json"
    cfg = json.loads(cfg_path.read_text())
    cfg["rules"].update(max_rounds=1, timeout_per_turn_seconds=60)
    cfg_path.write_text(json.dumps(cfg))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               ROUNDTABLE_BENCH_FAULT="0:engine_load:sleep15", ROUNDTABLE_COLLECTIVE_TIMEOUT_S="10")
    r = subprocess.run([sys.executable, "-m", "theroundtaible_amd", "discuss", "Laad traag", "--no-read-codebase",
                        "--choice", "4"], capture_output=True, text=True, timeout=400, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    sessions = os.listdir(tmp_path / ".roundtable" / "sessions")
    disc = (tmp_path / ".roundtable" / "sessions" / sessions[0] / "discussion.md").read_text()
    assert "Round 1 — Groot" in disc and "Round 1 — Klein" in disc, disc[:2000]
