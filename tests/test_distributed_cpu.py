"""Multi-process paths on CPU with gloo: TP equivalence, C1 token exchange, SPMD bench."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, model, q, overrides=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
        from theroundtaible_amd.parallel.tp import TPInfo
        tp = TPInfo(size=world, rank=rank, group=dist.group.WORLD)
        e = Engine(EngineConfig(model=model, device="cpu", dtype="fp32", num_blocks=64, weights="random-full:9",
                                model_overrides=dict(overrides or {})), tp)
        ids = e.encode_prompt("tensor parallel knight over xGMI")
        logits = e.prefill([(e.kv.seq("k"), ids)])
        out = e.run_turns([Turn("k2", "tensor parallel", SamplingParams(temperature=0, max_new_tokens=6,
                                                                        ignore_eos=True, stop_on_consensus=False))])[0]
        # greedy decode took the C3 (value, id) all-gather, not the full-logit gather
        assert getattr(tp, "c3_greedy_calls", 0) >= 5, "distributed greedy argmax not used"
        if rank == 0:
            q.put((logits.tolist(), out.ids))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model,tp,overrides", [("tiny-llama", 2, None), ("tiny-gpt2", 2, None),
                                                 ("tiny-llama", 4, {"n_kv_heads": 4}),
                                                 ("tiny-llama", 4, None),      # 2 KV heads: replicated
                                                 ("tiny-qwen", 2, None)])      # q/k/v bias sharded with the heads
def test_tp_matches_tp1(model, tp, overrides):
    """TP=2/4 forward + greedy decode equal TP=1; the TP decode samples
    greedily with the per-rank argmax + (value, id) all-gather (C3), so identical tokens show the
    distributed argmax matches the full-vocab one."""
    from theroundtaible_amd.engine import Engine, EngineConfig, SamplingParams, Turn
    e = Engine(EngineConfig(model=model, device="cpu", dtype="fp32", num_blocks=64, weights="random-full:9",
                            model_overrides=dict(overrides or {})))
    ids = e.encode_prompt("tensor parallel knight over xGMI")
    ref_logits = e.prefill([(e.kv.seq("k"), ids)])
    ref_ids = e.run_turns([Turn("k2", "tensor parallel", SamplingParams(temperature=0, max_new_tokens=6,
                                                                        ignore_eos=True, stop_on_consensus=False))])[0].ids
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, tp, port, model, q, overrides)) for r in range(tp)]
    for p in procs:
        p.start()
    logits, got_ids = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.allclose(torch.tensor(logits), ref_logits, atol=1e-3, rtol=1e-3)
    assert got_ids == ref_ids


def _exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.parallel.cluster import Cluster
        from theroundtaible_amd.parallel.exchange import exchange_token_ids
        c = Cluster(rank=rank, world=world, backend="gloo", cpu_group=dist.group.WORLD)
        mine = [(rank * 10 + i, list(range(rank + i + 1))) for i in range(rank + 1)]
        got = exchange_token_ids(c, mine, "cpu")
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def _static_exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.knights.base import TurnRequest, TurnResult
        from theroundtaible_amd.knights.distributed import DistributedPool, RemoteKnight
        from theroundtaible_amd.parallel.cluster import Cluster
        c = Cluster(rank=rank, world=world, backend="gloo", cpu_group=dist.group.WORLD)

        class Echo:   # local backend: replies with rank-dependent ids (rank 2's overflow the static width)
            def __init__(self, n):
                self.n = n

            def group_key(self):
                return self.n

            def max_source_chars(self):
                return None

            def execute_group(self, pairs, timeout_s):
                return [TurnResult("", list(range(12 if rank == 2 else 3 + rank)), "bpe", {}) for _ in pairs]

        placement = {f"K{r}": [r] for r in range(world)}
        pool = DistributedPool(c, placement, {f"K{rank}": Echo(rank)}, tokenizer=None, max_reply_tokens=8)
        ks = [RemoteKnight(pool, f"K{r}", f"K{r}", "x") for r in range(world)]
        res = pool.execute_round([(k, TurnRequest(k.name, "p")) for k in ks], 10.0)
        q.put((rank, [r.ids for r in res]))
    finally:
        dist.destroy_process_group()


def test_static_c1_exchange_with_overflow_fallback():
    """Static-shape async C1 all-gather; a rank whose reply exceeds the static width makes every
    rank join the shape-agreeing fallback, and all ranks still see every reply."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_static_exchange_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
    expect = [list(range(3)), list(range(4)), list(range(12))]
    for r in range(3):
        assert res[r] == expect


def test_token_exchange_ragged():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
    expect = {r * 10 + i: list(range(r + i + 1)) for r in range(3) for i in range(r + 1)}
    for r in range(3):
        assert res[r] == expect


def _bench(nproc, extra=()):
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--device", "cpu", "--model", "tiny-llama", "--steps", "2", "--warmup", "1", "--new-tokens", "8",
           "--temperature", "0", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def test_spmd_bench_two_ranks():
    out = _bench(2, ("--scaling", "weak"))
    assert out["n_gpus"] == 2 and out["config"]["knights"] == 6 and out["config"]["tables"] == 2
    assert out["detail"]["decode_tokens"] == 6 * 8 * 2
    assert out["value"] > 0 and out["scaling"] == "weak"


@pytest.mark.parametrize("nproc", [4, 8])
def test_spmd_bench_scaling_world_sizes(nproc):
    """The driver's scaling run (N = 4, 8 ranks) on the gloo/CPU path: 3 knights per rank, one
    table per rank sharing its prefix KV (default packed placement), every table's responses
    all-gathered to every rank in the C1 exchange."""
    out = _bench(nproc, ("--scaling", "weak"))
    assert out["n_gpus"] == nproc and out["config"]["tables"] == nproc and out["config"]["knights"] == 3 * nproc
    assert out["detail"]["decode_tokens"] == 3 * nproc * 8 * 2 and out["detail"]["failed_turns"] == 0
    assert out["config"]["placement"] == "packed" and out["config"]["prompt_layout"] == "shared"


def test_spmd_bench_striped_append_layout():
    """Round-1 placement and layout: knights of a table on different ranks, private KV."""
    out = _bench(4, ("--scaling", "weak", "--placement", "striped", "--layout", "append"))
    assert out["config"]["tables"] == 4 and out["detail"]["failed_turns"] == 0
    assert out["detail"]["decode_tokens"] == 3 * 4 * 8 * 2


def test_cli_discuss_under_torchrun_with_tp_knight(tmp_path):
    """`torchrun -m theroundtaible_amd discuss` (SPMD): one knight per rank plus a TP=2 knight
    spanning both ranks; rank 0 writes the session, every knight's turn lands in it."""
    cfg = {"version": "1.0", "project": "spmd", "language": "nl",
           "knights": [{"name": "Alfa", "adapter": "local-llm-alfa", "capabilities": ["x"], "priority": 1},
                       {"name": "Beta", "adapter": "local-llm-beta", "capabilities": ["x"], "priority": 2},
                       {"name": "Groot", "adapter": "local-llm-groot", "capabilities": ["x"], "priority": 3}],
           "rules": {"max_rounds": 2, "consensus_threshold": 9, "timeout_per_turn_seconds": 300,
                     "escalate_to_user_after": 5, "auto_execute": False, "ignore": [".git"],
                     "round_mode": "sequential"},
           "chronicle": ".roundtable/chronicle.md",
           "engine": {"default_model": "tiny-llama", "weights": "random-full:4", "max_new_tokens": 6,
                      "ignore_eos": True, "temperature": 0.0},
           "adapter_config": {"local-llm-alfa": {"engine": {"gpus": [0]}},
                              "local-llm-beta": {"engine": {"gpus": [1]}},
                              "local-llm-groot": {"engine": {"gpus": [0, 1], "tp": 2}}}}
    os.makedirs(tmp_path / ".roundtable" / "sessions")
    (tmp_path / ".roundtable" / "config.json").write_text(json.dumps(cfg))
    (tmp_path / ".roundtable" / "chronicle.md").write_text("# Chronicle\n")
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={port}", "-m", "theroundtaible_amd", "--quiet",
           "discuss", "SPMD onderwerp", "--no-read-codebase", "--choice", "4"]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    sessions = os.listdir(tmp_path / ".roundtable" / "sessions")
    assert len(sessions) == 1                                   # only rank 0 wrote into the project
    disc = (tmp_path / ".roundtable" / "sessions" / sessions[0] / "discussion.md").read_text()
    for name in ("Alfa", "Beta", "Groot"):
        assert disc.count(name) >= 2, name                       # both rounds, every knight (TP knight too)


def test_spmd_bench_tp2():
    """bench.py --tp 2 on 2 gloo ranks: one TP=2 group hosts the table's knights."""
    out = _bench(2, ("--tp", "2", "--knights-per-table", "2", "--knights-per-gpu", "2"))
    assert out["config"]["knights"] == 2 and "tp2" in out["config"]["parallelism"]
    assert out["detail"]["decode_tokens"] == 2 * 8 * 2


@pytest.mark.parametrize("nproc", [2, 4])
def test_strong_scaling_bench_one_table_tp(nproc):
    """The default ``--scaling strong``: ONE 3-knight table whose engine is tensor-parallel over
    all N ranks — the same discussion at every N, so ms/round is the
    BASELINE wall-clock curve; tiny-llama's 2 KV heads are replicated at tp 4."""
    out = _bench(nproc)
    assert out["scaling"] == "strong" and out["n_gpus"] == nproc
    assert out["config"]["tables"] == 1 and out["config"]["knights"] == 3
    assert out["config"]["parallelism"] == f"tp{nproc}" and out["config"]["tp"] == nproc
    assert out["detail"]["decode_tokens"] == 3 * 8 * 2 and out["detail"]["failed_turns"] == 0
    # the cost-model prediction rides along only for the configuration it was measured at
    assert out["detail"]["prediction"]["available"] is False


def test_strong_prediction_matches_cost_model_table():
    """bench.py's per-run prediction (detail.prediction) is the tools/tp_cost.py curve: the
    simulated rank-0 compute of that tp + 2L K9 calls and one gather per step + prefill rings."""
    from theroundtaible_amd.parallel.costmodel import load_simulated, strong_round_ms
    for n, want in ((2, 1270), (4, 949), (8, 814)):       # profiles/r06/tp_cost_model.md, K9 5 us
        sim = load_simulated(n)
        assert sim is not None and sim["config"]["tp"] == n
        assert abs(strong_round_ms(sim, n, 5.0, 9.5) - want) < 1.0
    one = load_simulated(1)
    assert strong_round_ms(one, 1, 5.0, 9.5) == one["ms_per_round"]
    # a fused all-reduce that saves s us per call removes 2L x s per step
    sim8 = load_simulated(8)
    d = strong_round_ms(sim8, 8, 8.0, 9.5) - strong_round_ms(sim8, 8, 8.0, 9.5, fused_saving_us=3.0)
    assert abs(d - 512 * 2 * 32 * 3.0 / 1e3) < 1e-6


def test_strong_scaling_matches_single_rank_tokens():
    """Greedy tokens of the strong-scaled table at tp 2 equal the 1-rank run (same table, same
    seed): the tensor-parallel engine changes the speed of the discussion, not its content."""
    one = _bench_single(("--temperature", "0", "--weights", "random-full:5"))
    two = _bench(2, ("--weights", "random-full:5"))
    assert two["detail"]["decode_tokens"] == one["detail"]["decode_tokens"]
    assert two["detail"]["transcript_sha"] == one["detail"]["transcript_sha"]


def _bench_single(extra=()):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--model", "tiny-llama", "--steps", "2",
           "--warmup", "1", "--new-tokens", "8", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_bench_gpus_flag_self_launches_ranks():
    """`python bench.py --gpus 4` without a launcher starts 4 ranks itself (child torchrun) and
    reports them — never a silent 1-GPU run. Default strong scaling: one table
    of 3 knights on a tp4 engine."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--device", "cpu", "--model", "tiny-llama",
           "--steps", "1", "--warmup", "1", "--new-tokens", "4", "--temperature", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 4 and out["detail"]["world"] == 4
    assert out["config"]["tables"] == 1 and out["config"]["knights"] == 3 and out["config"]["parallelism"] == "tp4"


def test_bench_rejects_world_mismatch():
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "3",
           "--device", "cpu", "--model", "tiny-llama", "--steps", "1", "--warmup", "0", "--new-tokens", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="1"),
                       cwd=ROOT)
    assert r.returncode != 0 and "refusing" in (r.stdout + r.stderr)


def test_bench_consensus_round_variant():
    """bench.py --consensus-round K: scripted consensus ends the table in round K (inside the
    timed region); forced tail tokens are reported apart from decoded ones."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--model", "tiny-llama", "--steps", "2",
           "--warmup", "1", "--new-tokens", "8", "--consensus-round", "3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    d = out["detail"]
    assert d["consensus_reached"] == 1 and d["consensus_round"] == 3
    assert d["decode_tokens"] == 3 * 8 * 2 and d["forced_tokens"] > 0


def _overlap_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from theroundtaible_amd.parallel.cluster import Cluster
        from theroundtaible_amd.parallel.exchange import TokenExchange
        c = Cluster(rank=rank, world=world, backend="gloo", cpu_group=dist.new_group(backend="gloo"))
        ex = TokenExchange(c, rows=1, width=16, device="cpu")
        order = []
        ex.start([(rank, [rank] * (rank + 2))])          # token all-gather in flight ...
        order.append("started")
        meta = c.all_gather_object({"rank": rank})       # ... while the metadata round runs
        order.append("metadata")
        got = ex.wait()
        order.append("tokens")
        q.put((rank, order, [m["rank"] for m in meta], got))
    finally:
        dist.destroy_process_group()


def test_c1_token_gather_overlaps_metadata_round():
    """C1 ordering (knights/distributed.py): the static token all-gather is issued first and
    left in flight, the gloo metadata round completes, then the tokens are collected."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (o, m, g)) for r, o, m, g in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        order, meta, got = res[r]
        assert order == ["started", "metadata", "tokens"] and meta == [0, 1]
        assert got == {0: [0, 0], 1: [1, 1, 1]}


def _tp_project(tmp_path, knights_engine):
    cfg = {"version": "1.0", "project": "spmd", "language": "nl",
           "knights": [{"name": n, "adapter": f"local-llm-{n.lower()}", "capabilities": ["x"], "priority": i + 1}
                       for i, n in enumerate(knights_engine)],
           "rules": {"max_rounds": 1, "consensus_threshold": 9, "timeout_per_turn_seconds": 300,
                     "escalate_to_user_after": 5, "auto_execute": False, "ignore": [".git"]},
           "chronicle": ".roundtable/chronicle.md",
           "engine": {"default_model": "tiny-llama", "weights": "random-full:4", "max_new_tokens": 6,
                      "ignore_eos": True, "temperature": 0.0, "device": "cpu"},
           "adapter_config": {f"local-llm-{n.lower()}": {"engine": eng} for n, eng in knights_engine.items()}}
    os.makedirs(tmp_path / ".roundtable" / "sessions")
    (tmp_path / ".roundtable" / "config.json").write_text(json.dumps(cfg))
    (tmp_path / ".roundtable" / "chronicle.md").write_text("# Chronicle\n")


def test_plain_cli_discuss_launches_tp_ranks(tmp_path):
    """a plain ``python -m theroundtaible_amd discuss`` (no torchrun) with a
    ``tp: 2`` knight starts the 2 ranks itself before any device call and the knight really runs
    tensor-parallel: metrics.jsonl records tp=2 for its turns; rc 0; one session written."""
    _tp_project(tmp_path, {"Groot": {"tp": 2}, "Klein": {}})
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-m", "theroundtaible_amd", "discuss", "TP onderwerp", "--no-read-codebase",
                        "--choice", "4"], capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "Launching 2 ranks" in r.stderr
    sessions = os.listdir(tmp_path / ".roundtable" / "sessions")
    assert len(sessions) == 1
    recs = [json.loads(l) for l in (tmp_path / ".roundtable" / "sessions" / sessions[0] / "metrics.jsonl")
            .read_text().splitlines() if l.strip()]
    tps = {m["knight"]: m.get("tp") for m in recs if "knight" in m}
    assert tps == {"Groot": 2, "Klein": 1}, tps


def test_tp_knight_outside_a_launcher_is_refused(tmp_path):
    """The in-process backend factory never degrades a tp > 1 knight to tp 1."""
    from theroundtaible_amd.config import load_config
    from theroundtaible_amd.errors import ConfigError
    from theroundtaible_amd.knights.registry import BackendFactory
    _tp_project(tmp_path, {"Groot": {"tp": 2}})
    with pytest.raises(ConfigError):
        BackendFactory(load_config(str(tmp_path))).create("local-llm-groot")


def test_ranks_needed_from_placement(tmp_path):
    from theroundtaible_amd.config import load_config
    from theroundtaible_amd.parallel.launch import ranks_needed
    _tp_project(tmp_path, {"A": {"tp": 4}, "B": {"gpus": [5]}, "C": {}})
    n, why, cpu = ranks_needed(load_config(str(tmp_path)))
    assert n == 6 and "A tp=4" in why and cpu


def test_c1_overlaps_speculative_prefill_striped():
    """in a striped table (knights on different ranks) each rank prefills what it
    already knows of the next round's shared prompt (its own finished entries at the head of the
    speaking order) WHILE the C1 all-gather of the other ranks' replies is in flight; the next
    round keeps that KV by LCP. Pinned: the order c1_start < speculate < c1_wait, speculative
    tokens were prefilled, and the transcripts equal a run without speculation."""
    on = _bench(2, ("--scaling", "weak", "--placement", "striped", "--temperature", "0.8"))
    env_off = dict(os.environ, ROUNDTABLE_C1_SPECULATE="0")
    old = os.environ.get("ROUNDTABLE_C1_SPECULATE")
    os.environ["ROUNDTABLE_C1_SPECULATE"] = "0"
    try:
        off = _bench(2, ("--scaling", "weak", "--placement", "striped", "--temperature", "0.8"))
    finally:
        if old is None:
            os.environ.pop("ROUNDTABLE_C1_SPECULATE", None)
        else:
            os.environ["ROUNDTABLE_C1_SPECULATE"] = old
    del env_off
    d_on, d_off = on["detail"], off["detail"]
    assert d_on["failed_turns"] == 0 and d_off["failed_turns"] == 0
    assert d_on["c1_overlap_order_ok"] is True
    assert d_on["c1_speculations_rank0"] > 0 and d_on["speculative_prefill_tokens_rank0"] > 0
    # every speculated token was the real next prompt's (kept by LCP; none rolled back) — except
    # in the last round, whose speculation no later turn consumes
    assert 0 < d_on["speculative_kept_tokens_rank0"] <= d_on["speculative_prefill_tokens_rank0"]
    assert d_off["c1_speculations_rank0"] == 0 and d_off["speculative_prefill_tokens_rank0"] == 0
    assert d_on["transcript_sha"] == d_off["transcript_sha"]
    # the speculated KV was reused: the turns themselves prefilled fewer tokens
    assert d_on["prefill_tokens"] < d_off["prefill_tokens"]


def test_strong_scaling_sampled_decode_tp2():
    """Sampled (temperature 0.7, top-p 0.95) tensor-parallel decode, the driver bench's setting:
    logit shards all-gathered in ONE all_gather_into_tensor and sampled on the full row, every
    rank drawing the same token."""
    out = _bench(2, ("--temperature", "0.7"))
    assert out["config"]["parallelism"] == "tp2" and out["detail"]["failed_turns"] == 0
    assert out["detail"]["decode_tokens"] == 3 * 8 * 2


def test_strong_prediction_sequential_rounds_count_every_speaker():
    """Sequential rounds (reference semantics): each of the table's speakers decodes its own
    turn at B = 1, so a round carries knights x new_tokens decode steps, each with 2L K9 calls
    and one logits gather (the cost model now covers this mode)."""
    from theroundtaible_amd.parallel.costmodel import strong_round_ms
    sim = {"config": {"model": "llama3-8b", "new_tokens_per_turn": 512, "knights_per_table": 3,
                      "round_mode": "sequential"},
           "ms_per_round": 1000.0, "steps": 20, "detail": {"prefill_tokens": 20 * 1800}}
    par = dict(sim, config=dict(sim["config"], round_mode="parallel"))
    d_seq = strong_round_ms(sim, 8, 8.0, 9.5) - 1000.0
    d_par = strong_round_ms(par, 8, 8.0, 9.5) - 1000.0
    decode = 512 * (2 * 32 * 8.0 + 9.5) / 1e3
    # the prefill ring all-reduces carry the same bytes in both modes; sequential pays their
    # fixed per-call cost once per speaker
    assert abs((d_seq - d_par) - (2 * decode + 2 * 2 * 32 * 0.02)) < 0.01
    assert d_par > decode


def test_rehearsal_ranks_sharing_a_gpu_cap_their_hardware_queues(monkeypatch):
    """8 gloo rehearsal ranks on one card map at most 16 hardware queues together (2 each; the
    4-queue default hung the captured K9 warm-up, profiles/r05/rehearsal/); 4 ranks keep HIP's
    default, as do a lower value already set, RCCL worlds and one rank per card."""
    from theroundtaible_amd.parallel import cluster
    monkeypatch.setattr(cluster.torch.cuda, "device_count", lambda: 1)
    env = {"ROUNDTABLE_DIST_BACKEND": "gloo"}
    assert cluster.limit_shared_gpu_queues(env, 4) is None and "GPU_MAX_HW_QUEUES" not in env
    assert cluster.limit_shared_gpu_queues(env, 8) == 2 and env["GPU_MAX_HW_QUEUES"] == "2"
    env = {"ROUNDTABLE_DIST_BACKEND": "gloo", "GPU_MAX_HW_QUEUES": "4"}     # as the GPU boxes export it
    assert cluster.limit_shared_gpu_queues(env, 8) == 2 and env["GPU_MAX_HW_QUEUES"] == "2"
    env = {"ROUNDTABLE_DIST_BACKEND": "gloo", "GPU_MAX_HW_QUEUES": "1"}     # never raised
    assert cluster.limit_shared_gpu_queues(env, 8) is None and env["GPU_MAX_HW_QUEUES"] == "1"
    assert cluster.limit_shared_gpu_queues({}, 8) is None               # RCCL: one rank per card
    monkeypatch.setattr(cluster.torch.cuda, "device_count", lambda: 8)
    assert cluster.limit_shared_gpu_queues({"ROUNDTABLE_DIST_BACKEND": "gloo"}, 8) is None


def test_rehearsal_cu_split_gives_each_sharing_rank_a_disjoint_slice(monkeypatch):
    """ROUNDTABLE_REHEARSAL_CU_SPLIT=1: ranks sharing one card get disjoint, equal CU masks (the
    mask HIP reads at start-up); off by default, and nothing for one rank per card."""
    from theroundtaible_amd.parallel import cluster
    monkeypatch.setattr(cluster.torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(cluster, "_card_cus", lambda default=256: 256)
    monkeypatch.delenv("ROUNDTABLE_REHEARSAL_CU_SPLIT", raising=False)
    monkeypatch.delenv("ROC_GLOBAL_CU_MASK", raising=False)
    assert cluster.rehearsal_cu_split(4, 1) is None and "ROC_GLOBAL_CU_MASK" not in os.environ
    monkeypatch.setenv("ROUNDTABLE_REHEARSAL_CU_SPLIT", "1")
    masks = [int(cluster.rehearsal_cu_split(4, r), 16) for r in range(4)]
    assert all(bin(m).count("1") == 64 for m in masks)
    assert sum(masks) == (1 << 256) - 1 and all(a & b == 0 for i, a in enumerate(masks) for b in masks[i + 1:])
    monkeypatch.setattr(cluster.torch.cuda, "device_count", lambda: 4)
    monkeypatch.delenv("ROC_GLOBAL_CU_MASK", raising=False)
    assert cluster.rehearsal_cu_split(4, 2) is None and "ROC_GLOBAL_CU_MASK" not in os.environ
