#!/usr/bin/env python3
"""Roundtable benchmark: wall-clock per round + aggregate knight tokens/s (BASELINE.json metric).

Workload (one "step" = one complete discussion round):
  * knights are Llama-3-8B (bf16, random-init weights: there are no checkpoints), 3 per
    table, a table = one 3-knight ``discuss`` (BASELINE config 2 / metric "3-knight discuss");
  * ``--scaling strong`` (default): ONE table whatever N is — its 3 knights batched in one
    decode hipGraph on ONE engine that is tensor-parallel over all N GPUs (Megatron split,
    split-K shard GEMMs, K9 one-shot all-reduce over xGMI, vocab-parallel lm_head). Total work
    is fixed, so ``ms_per_round`` at N = 1/2/4/8 is the BASELINE wall-clock curve of the same
    discussion (the reference's per-round cost is its sequential knight loop,
    /root/reference/src/orchestrator.ts:347-536);
  * ``--scaling weak``: N GPUs host N tables (3N knights), 3 knights per GPU group.
    ``--placement packed``: table t lives on GPU t, so its knights share one copy of the
    discussion's KV (``shared`` layout); every rank still runs every table's orchestrator
    (SPMD) and each round's responses are all-gathered over RCCL (C1). ``striped``: knight j
    of table t on rank (3t + j) mod N, every response crossing xGMI;
  * ``--simulate-tp N`` (cost model only, never a measurement of N GPUs): one process computes
    rank 0's shard of a tp=N engine with every collective replaced by a local no-op
    (parallel/tp.py SimulatedTP); tools/tp_cost.py adds the measured collective latencies;
  * ``parallel`` round mode, ``shared`` prompt layout (``--layout append`` is the
    round-1 layout), the real orchestrator (prompt assembly, consensus parse,
    discussion.md/metrics writes) inside the timed region;
  * fixed ``--new-tokens`` per turn with EOS ignored (random weights never emit a
    consensus block; BASELINE.md measurement protocol).

The reference publishes no numbers (BASELINE.json "published": {}), so ``vs_baseline`` is
null; ``reference_bound_ms_per_round`` records its implied upper bound (3 knights x the
120 s per-turn timeout, sequential) for context.

Launch: ``python bench.py --gpus 1`` or, for N > 1,
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

TOPIC = ("Hoe structureren we de resident KV-cache van elke knight zodat een discussie van vijf rondes "
         "volledig in HBM blijft, en welke consistentie-garanties geven we bij een crash midden in een ronde?")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3, help="timed rounds")
    p.add_argument("--warmup", type=int, default=1, help="untimed rounds (round 1 includes the initial prefill)")
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--knights-per-gpu", type=int, default=None,
                   help="knights hosted per GPU group (a TP group when --tp > 1); default: the whole table "
                        "(strong) / 3 (weak). BASELINE config 5 = --tp 4 --knights-per-table 2 --knights-per-gpu 1 "
                        "on 8 GPUs: two disjoint TP=4 groups, one knight each")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                   help="strong (default): one 3-knight table, one engine tensor-parallel over all N GPUs; "
                        "weak: N tables, one GPU group each")
    p.add_argument("--tp", type=int, default=0,
                   help="tensor-parallel degree of every knight (0 = N under --scaling strong, 1 under weak; "
                        "BASELINE config 5: 4)")
    p.add_argument("--simulate-tp", type=int, default=0,
                   help="COST MODEL ONLY: one process runs rank 0's shard of a tp=N engine, collectives replaced "
                        "by local no-ops (the output is labelled simulated)")
    p.add_argument("--sim-k9-us", type=float, default=5.0,
                   help="--simulate-tp: device-side stand-in latency of each all-reduce (a spin kernel holding the "
                        "K9 launch's CUs, inside the captured graph); 0 = collectives free (round-4 compute-only records)")
    p.add_argument("--sim-gather-us", type=float, default=9.5,
                   help="--simulate-tp: the same for the vocab-parallel logits gather (0 = free)")
    p.add_argument("--knights-per-table", type=int, default=3)
    p.add_argument("--new-tokens", type=int, default=512, help="decode tokens per knight turn")
    p.add_argument("--temperature", type=float, default=0.7)
    p.add_argument("--top-p", type=float, default=0.95)
    p.add_argument("--round-mode", default="parallel", choices=["parallel", "sequential"],
                   help="parallel: all knights of a round decode as one batch; sequential: reference "
                        "semantics (speakers in order, each sees the earlier speakers of the round)")
    p.add_argument("--layout", default="shared", choices=["shared", "append", "reference"],
                   help="prompt layout; 'shared' (default) keeps ONE copy of a table's common prefix KV per GPU, "
                        "read once per decode step for all of the table's knights there (grouped K3)")
    p.add_argument("--c1-events", default="",
                   help="write each rank's C1 event log (name, CLOCK_MONOTONIC ns) to <path>.r<rank>.json")
    p.add_argument("--placement", default="packed", choices=["packed", "striped"],
                   help="packed (default): a table's knights share one GPU group (batched decode + shared prefix "
                        "KV); striped: knight j of table t on group (kpt*t + j) mod groups (every response "
                        "crosses xGMI, no KV sharing)")
    p.add_argument("--weights", default="random:1234",
                   help="random:<seed> (per-rank shards, fast) | random-full:<seed> (unsharded tensors split per rank: "
                        "a tp=N run has exactly the tp=1 weights; tests) | a checkpoint path")
    p.add_argument("--layers", type=int, default=None,
                   help="rehearsal only: override the model's layer count (reported in config.model)")
    p.add_argument("--weight-residency", default="auto", choices=["auto", "dual", "shuffled"])
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--kv-fraction", type=float, default=0.85,
                   help="fraction of free HBM for the KV pool (lower it when ranks share a GPU)")
    p.add_argument("--max-kv-tokens", type=int, default=None, help="cap the KV pool (tokens per engine)")
    p.add_argument("--device", default=None, help="override device (cpu for a plumbing run)")
    p.add_argument("--consensus-round", type=int, default=0,
                   help="scripted consensus (knights/script.py): after the free --new-tokens every knight's reply "
                        "ends in a forced consensus JSON scoring 6, then 9 in this round, so the tables reach "
                        "consensus and stop there (0 = off; use warmup + steps to end inside the timed region)")
    p.add_argument("--out", default=None, help="also write the JSON line to this file")
    p.add_argument("--stage-timeout", type=float, default=240.0,
                   help="seconds any stage (a round, a capture) may take on any rank, and the process-group "
                        "collective timeout; past it rank 0 prints the failure line and every rank exits")
    p.add_argument("--init-timeout", type=float, default=900.0,
                   help="the same for start-up (rendezvous, weights, K9 creation: a fresh box pages torch in)")
    p.add_argument("--write-calibration", default=None,
                   help="(N > 1) write the node's measured K9 latency / fused saving as a cost-model calibration "
                        "JSON (parallel/costmodel.py default_calibration, $ROUNDTABLE_CALIBRATION)")
    return p.parse_args()


def _self_launch(args) -> int:
    """``--gpus N`` (N > 1) outside a launcher: start the N ranks as a CHILD torchrun (before this
    process touches the GPU), forward its output and exit with its code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    if args.device != "cpu":
        from theroundtaible_amd.parallel.cluster import limit_shared_gpu_queues
        limit_shared_gpu_queues(env, args.gpus)     # gloo rehearsal ranks sharing one card
    return subprocess.run(cmd, env=env).returncode


def _overlap_order_ok(events) -> bool:
    """Every speculative prefill ran while a C1 all-gather was in flight (after its start,
    before its wait)."""
    open_ = False
    for e in events:
        if e == "c1_start":
            open_ = True
        elif e == "c1_wait":
            open_ = False
        elif e == "speculate" and not open_:
            return False
    return True


def _predict(args, T: int, engine) -> dict:
    """The cost model's prediction for THIS strong-scaling run (profiles/r03/tp_cost_model.md),
    re-evaluated with the K9 latency / fused saving / gather cost the engine just measured on the
    node's own links — so the driver's N-GPU record carries prediction and measurement side by
    side. Only for the configuration the simulated compute was measured at."""
    from theroundtaible_amd.parallel.costmodel import Calibration, load_simulated, strong_round_ms
    simr = load_simulated(T, args.round_mode)
    if simr is None:
        return {"available": False, "reason": f"no simulated tp{T} {args.round_mode} record (parallel/calib/)"}
    c = simr["config"]
    same = (c["model"] == args.model and c["new_tokens_per_turn"] == args.new_tokens
            and c["knights_per_table"] == args.knights_per_table and c["round_mode"] == args.round_mode
            and c["prompt_layout"] == args.layout and simr["steps"] == args.steps and simr["warmup"] == args.warmup)
    if not same:
        return {"available": False, "reason": "configuration differs from the simulated run"}
    os_ = getattr(engine.tp, "oneshot", None)
    cal = Calibration()
    k9 = os_.latency_us if os_ is not None and os_.latency_us else cal.ar_us
    saving = os_.fused_saving_us if os_ is not None and os_.fused and os_.fused_saving_us else 0.0
    gather = cal.gather_us    # one-shot gather as measured on one GPU; the probe keeps the faster of it / RCCL
    return {"available": True, "simulated_compute_ms_per_round": simr["ms_per_round"],
            "k9_us": k9, "fused_saving_us": saving, "gather_us": gather,
            "predicted_ms_per_round": round(strong_round_ms(simr, T, k9, gather, saving), 1)}


def _failure_line(args, world: int, rec: dict) -> dict:
    """Rank 0's one JSON line for a run that could not finish (utils/failsafe.py): the stage and
    rank that failed instead of a measurement."""
    return {"metric": f"aggregate knight tokens/sec ({args.knights_per_table}-knight discuss, {args.round_mode} rounds)",
            "value": None, "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": None, "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "bf16" if args.device != "cpu" else "fp32", "data": "synthetic prompts, random-init weights",
            "config": {"model": args.model, "knights_per_table": args.knights_per_table, "round_mode": args.round_mode,
                       "prompt_layout": args.layout, "tp": args.tp or None},
            "error": rec.get("error"), "failed_stage": rec.get("failed_stage"), "failed_rank": rec.get("failed_rank"),
            "failures": rec.get("failures", [])}


def main() -> int:
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(args)
    from theroundtaible_amd.utils import failsafe
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    # every stage of this rank runs under a time limit, and any rank's failure ends the whole run
    # with ONE JSON line from rank 0 naming the stage: a wedged collective never
    # eats the driver's window in silence
    guard = failsafe.RunGuard(rank, world, lambda rec: print(json.dumps(_failure_line(args, world, rec)), flush=True),
                              default_s=args.stage_timeout,
                              limits={"start": args.init_timeout, "init": args.init_timeout,
                                      "engine_load": args.init_timeout, "k9_create": args.init_timeout}).start()
    try:
        rc = _run(args, failsafe)
    except BaseException as e:  # noqa: BLE001 - every failure becomes the run's JSON line
        guard.fail(failsafe.current_stage(), f"{type(e).__name__}: {e}")
        return 3
    guard.finish()
    return rc


def _run(args, failsafe) -> int:
    from theroundtaible_amd.utils.debug import apply_debug_env
    if apply_debug_env():
        print("bench: ROUNDTABLE_DEBUG=1 — kernels serialized, numbers are NOT performance data", file=sys.stderr)
    import torch
    from theroundtaible_amd.engine.engine import Engine, EngineConfig
    from theroundtaible_amd.engine.sampler import SamplingParams
    from theroundtaible_amd.knights.distributed import DistributedPool, RemoteKnight
    from theroundtaible_amd.knights.engine_backend import EngineBackend
    from theroundtaible_amd.orchestrator import Orchestrator, RunOptions, run_tables_parallel, run_tables_sequential
    from theroundtaible_amd.parallel.cluster import init_cluster
    from theroundtaible_amd.types import RoundtableConfig

    failsafe.set_stage("init")
    # collectives time out a little after the stage guard fires (utils/failsafe.py), so a stall is
    # reported by the guard's JSON line rather than by a process-group abort; <= 300 s by default
    cl = init_cluster(prefer_gpu=args.device != "cpu", timeout_s=int(args.stage_timeout) + 30)
    N = cl.world
    if N != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {N} rank(s) joined (WORLD_SIZE); refusing to "
                         f"report a {N}-GPU run as {args.gpus}")
    device = args.device or cl.device
    kpt = args.knights_per_table
    sim = max(0, args.simulate_tp)
    if sim and N != 1:
        raise SystemExit("--simulate-tp runs ONE process (it models one rank of a tp group)")
    T = args.tp if args.tp > 0 else (N if args.scaling == "strong" else 1)
    if args.knights_per_gpu is None:
        # strong: one table on one TP group, every GPU of the group hosts all of the table's knights
        args.knights_per_gpu = kpt if args.scaling == "strong" else 3
    if N % T:
        raise SystemExit(f"--tp {T} must divide the {N} launched GPUs")
    from theroundtaible_amd.models.config import get_config
    mc = get_config(args.model, **({"n_layers": args.layers} if args.layers else {}))
    if T > 1 and (mc.n_heads % T or mc.ffn % T or (mc.n_kv_heads % T and T % mc.n_kv_heads)):
        raise SystemExit(f"{args.model} ({mc.n_heads} heads, {mc.n_kv_heads} KV heads, FFN {mc.ffn}) "
                         f"does not split over tp={T}")
    n_groups = N // T                      # GPU groups; a knight lives on one group (T ranks)
    total_knights = args.knights_per_gpu * n_groups
    n_tables = max(1, total_knights // kpt)
    base_names = ["Claude", "Gemini", "GPT", "Mistral", "Llama", "Qwen", "Phi", "Falcon"]
    group_ranks = [list(range(g * T, (g + 1) * T)) for g in range(n_groups)]
    placement = {}
    tables = []
    for t in range(n_tables):
        knights = []
        for j in range(kpt):
            name = f"{base_names[j % len(base_names)]}-{t}"
            slot = (t * kpt + j) // max(1, args.knights_per_gpu) if args.placement == "packed" else kpt * t + j
            placement[name] = group_ranks[slot % n_groups]
            knights.append({"name": name, "adapter": f"local-llm-{name.lower()}", "capabilities": ["architecture"],
                            "priority": j + 1})
        tables.append(knights)
    local_names = [n for n, ranks in placement.items() if cl.rank in ranks]

    failsafe.set_stage("tp_groups")
    tp = None
    if sim > 1:
        from theroundtaible_amd.parallel.tp import SimulatedTP
        tp = SimulatedTP(sim, comm_us=args.sim_k9_us or None, gather_us=args.sim_gather_us or None)
        if tp.comm_us or tp.gather_us:
            tp.calibrate_stand_in()      # calibrate the stand-in's launch cost before any capture
    elif T > 1:
        import torch.distributed as dist
        from theroundtaible_amd.parallel.tp import TPInfo
        pgs = [dist.new_group(r) for r in group_ranks]   # collective: same order on every rank
        g = cl.rank // T
        tp = TPInfo(size=T, rank=cl.rank % T, group=pgs[g])
    failsafe.set_stage("engine_load")
    t_load = time.perf_counter()
    engine = Engine(EngineConfig(model=args.model, weights=args.weights, device=device,
                                 use_graphs=not args.no_graphs and device != "cpu",
                                 dtype="bf16" if device != "cpu" else "fp32",
                                 kv_cache_fraction=args.kv_fraction, max_kv_tokens=args.max_kv_tokens,
                                 weight_residency=args.weight_residency,
                                 model_overrides={"n_layers": args.layers} if args.layers else {}), tp)
    params = SamplingParams(temperature=args.temperature, top_p=args.top_p, max_new_tokens=args.new_tokens,
                            ignore_eos=True, stop_on_consensus=False, seed=7)
    import threading
    lock = threading.Lock()
    script = None
    if args.consensus_round:
        from theroundtaible_amd.knights.script import ConsensusScript
        script = ConsensusScript(free_tokens=args.new_tokens, scores=[6] * (args.consensus_round - 1) + [9],
                                 files=["NEW:docs/besluit.md"])
    local = {n: EngineBackend(n, f"local-llm-{n.lower()}", engine, params, lock, script=script) for n in local_names}
    pool = DistributedPool(cl, placement, local, engine.tokenizer, max_reply_tokens=args.new_tokens + 512)
    load_s = time.perf_counter() - t_load

    failsafe.set_stage("setup")
    rounds = args.warmup + args.steps
    workdir = tempfile.mkdtemp(prefix=f"rt-bench-r{cl.rank}-")
    orchs = []
    for t, knights in enumerate(tables):
        cfg = RoundtableConfig.from_dict({
            "version": "1.0", "project": "bench", "language": "nl", "knights": knights,
            "rules": {"max_rounds": rounds, "consensus_threshold": 9, "timeout_per_turn_seconds": 3600,
                      "escalate_to_user_after": rounds + 1, "auto_execute": False, "ignore": [".git"],
                      "round_mode": args.round_mode, "prompt_layout": args.layout},
            "chronicle": ".roundtable/chronicle.md", "adapter_config": {}})
        backends = {k["adapter"]: RemoteKnight(pool, k["name"], k["name"], k["adapter"]) for k in knights}
        # every rank runs every table (SPMD), but only the rank leading the table's first knight
        # writes its session files: per-rank host work stays one table's as N grows
        persist = placement[knights[0]["name"]][0] == cl.rank
        orchs.append(Orchestrator(cfg, backends, workdir, options=RunOptions(shuffle_seed=1000 + t,
                                                                             max_new_tokens=args.new_tokens,
                                                                             persist=persist),
                                  store_root=workdir))

    timing = {}

    def on_round(rnd: int, ms: float):
        failsafe.set_stage(f"round {rnd + 1}" if rnd < rounds else "report")
        if rnd == args.warmup:
            if device.startswith("cuda"):
                torch.cuda.synchronize()
            cl.barrier()
            timing["t0"] = time.perf_counter()
        if rnd == rounds or (args.consensus_round and rnd == args.consensus_round):
            if device.startswith("cuda"):
                torch.cuda.synchronize()
            cl.barrier()
            timing["t1"] = time.perf_counter()

    if args.warmup == 0:
        cl.barrier()
        timing["t0"] = time.perf_counter()
    runner = run_tables_parallel if args.round_mode == "parallel" else run_tables_sequential
    failsafe.set_stage("round 1")
    runner(orchs, [f"{TOPIC} (tafel {t})" for t in range(n_tables)], on_round=on_round)
    elapsed = cl.max_scalar(timing["t1"] - timing["t0"])
    last = min(rounds, args.consensus_round) if args.consensus_round else rounds
    timed = range(args.warmup + 1, last + 1)
    dec = pre = reused = forced = 0
    # engine time per timed round (parallel: the slowest turn of the round, turns of one engine
    # batch run together) vs the round's wall clock: the rest is host work (prompts, parse, files, C1)
    eng_ms, pre_ms, dec_ms = {}, {}, {}
    # (sequential rounds: the knights' turns run one after another, so their engine times add up)
    agg = (lambda a, b: a + b) if args.round_mode == "sequential" else max
    for o in orchs:
        for e in o.all_rounds:
            if e.round in timed:
                eng_ms[e.round] = agg(eng_ms.get(e.round, 0.0), float(e.metrics.get("turn_ms", 0.0)))
                pre_ms[e.round] = agg(pre_ms.get(e.round, 0.0), float(e.metrics.get("prefill_ms", 0.0)))
                dec_ms[e.round] = agg(dec_ms.get(e.round, 0.0), float(e.metrics.get("decode_ms", 0.0)))
    ctx = []     # each timed turn's context at its end (prompt + reply tokens) per knight
    for o in orchs:
        for e in o.all_rounds:
            if e.round in timed:
                ctx.append(int(e.metrics.get("prompt_tokens", 0)) + int(e.metrics.get("decode_tokens", 0))
                           + int(e.metrics.get("forced_tokens", 0)))
    for o in orchs:
        for e in o.all_rounds:
            if e.round in timed:
                dec += int(e.metrics.get("decode_tokens", 0))
                pre += int(e.metrics.get("prefill_tokens", 0))
                reused += int(e.metrics.get("reused_tokens", 0))
                forced += int(e.metrics.get("forced_tokens", 0))
    import hashlib
    h = hashlib.sha256()
    for o in orchs:
        for e in o.all_rounds:
            h.update(f"{e.round}|{e.knight}|{e.response}\n".encode())
    transcript_sha = h.hexdigest()[:16]
    failures = [f for o in orchs for f in o.failures]
    if failures:
        print(f"[rank {cl.rank}] {len(failures)} failed knight turns; first: {failures[0]}", file=sys.stderr, flush=True)
    n_timed = max(1, len(timed))
    exch = sum(pool.exchange_ms[-n_timed:]) / n_timed if pool.exchange_ms else 0.0
    ms_round = elapsed / n_timed * 1e3
    value = dec / elapsed if elapsed > 0 else 0.0
    ref_bound_ms = kpt * 120_000.0
    if n_tables == 1:
        metric = f"aggregate knight tokens/sec (one {kpt}-knight discuss, {args.round_mode} rounds)"
    else:
        metric = f"aggregate knight tokens/sec ({kpt}-knight discuss tables, {args.round_mode} rounds)"
    if sim and args.sim_k9_us:
        metric = (f"SIMULATED rank 0 of tp{sim}: shard compute + device-simulated collectives (all-reduce "
                  f"{args.sim_k9_us:g} us, gather {args.sim_gather_us:g} us per call) — " + metric)
    elif sim:
        metric = f"SIMULATED rank-0 compute of tp{sim} (no communication; cost model input) — " + metric
    if sim:
        parallelism = (f"simulated tp{sim} (rank 0 shard, collectives "
                       + (f"simulated on device: {args.sim_k9_us:g} us all-reduce, {args.sim_gather_us:g} us gather)"
                          if args.sim_k9_us else "elided)"))
    elif T == 1:
        parallelism = (f"knight-placement x{N} (tables {args.placement} over GPUs), C1 all-gather"
                       if N > 1 else "single GPU")
    elif n_groups == 1:
        parallelism = f"tp{T}"
    else:
        parallelism = f"tp{T} knights x{n_groups} groups, C1 all-gather + C2/C3 RCCL"
    out = {
        "metric": metric,
        "value": round(value, 2), "unit": "tokens/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_round, 2), "ms_per_round": round(ms_round, 2),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
        "reference_bound_ms_per_round": ref_bound_ms, "speedup_vs_reference_bound": round(ref_bound_ms / ms_round, 1),
        "dtype": "bf16" if device != "cpu" else "fp32", "data": "synthetic prompts, random-init weights",
        "config": {"model": args.model + (f" ({args.layers} layers, rehearsal)" if args.layers else ""),
                   "knights_per_table": kpt, "tables": n_tables, "knights": kpt * n_tables,
                   "knights_per_gpu": args.knights_per_gpu, "new_tokens_per_turn": args.new_tokens,
                   # seq_len = the longest context a knight's decode attends over in the timed
                   # rounds (prompt + reply); the decode length per turn is new_tokens_per_turn
                   "global_batch": kpt * n_tables, "seq_len": max(ctx, default=0),
                   "context_tokens_per_knight_mean": round(sum(ctx) / len(ctx)) if ctx else 0,
                   "context_tokens_per_knight_max": max(ctx, default=0),
                   "round_mode": args.round_mode, "prompt_layout": args.layout,
                   "placement": args.placement, "tp": sim or T,
                   "parallelism": parallelism},
        "detail": {"world": cl.world, "backend": cl.backend, "c1_ranks": cl.world if cl.distributed else 1,
                   "simulated_tp": sim or None,
                   "sim_comm": ({"all_reduce_us": args.sim_k9_us, "gather_us": args.sim_gather_us,
                                 "spin_launch_us": round(tp.stand_in_launch_us, 2) if getattr(tp, "stand_in_launch_us", None) else None,
                                 "stand_in_nodes_issued_at_capture_or_eagerly": getattr(tp, "sim_comm_calls", 0)}
                                if sim and args.sim_k9_us else None),
                   "k9_oneshot": bool(getattr(engine.tp, "oneshot", None)),
                   "k9_us": getattr(getattr(engine.tp, "oneshot", None), "latency_us", None),
                   "k9_fused_gemm_ar": bool(getattr(getattr(engine.tp, "oneshot", None), "fused", False)),
                   "k9_fused_saving_us": getattr(getattr(engine.tp, "oneshot", None), "fused_saving_us", None),
                   "k9_ll": getattr(getattr(engine.tp, "oneshot", None), "ll", None),
                   "k9_flag_us": getattr(getattr(engine.tp, "oneshot", None), "flag_latency_us", None),
                   "k9_ll_us": getattr(getattr(engine.tp, "oneshot", None), "ll_latency_us", None),
                   "k9_gather": bool(getattr(getattr(engine.tp, "oneshot", None), "gather_ok", False)),
                   "k9_gather_saving_us": getattr(getattr(engine.tp, "oneshot", None), "gather_saving_us", None),
                   "k9_resyncs": engine.stats.get("k9_resyncs", 0),
                   "failed_turns": len(failures), "transcript_sha": transcript_sha, "decode_tokens": dec, "prefill_tokens": pre, "reused_kv_tokens": reused,
                   "exchange_ms_per_round": round(exch, 3), "c1_skipped_batches": getattr(pool, "c1_skipped", 0),
                   "c1_device_assembled": pool.exchange.device_path if pool.exchange is not None else 0,
                   "speculative_prefill_tokens_rank0": engine.stats.get("speculative_tokens", 0),
                   "speculative_kept_tokens_rank0": engine.stats.get("speculative_kept", 0),
                   "c1_speculations_rank0": pool.events.count("speculate"),
                   "c1_overlap_order_ok": _overlap_order_ok(pool.events),
                   "engine_load_s": round(load_s, 2),
                   "resident_tokens_rank0": sum(s.length for s in engine.kv.seqs.values()),
                   "kv_blocks_used_rank0": engine.kv.num_blocks - engine.kv.alloc.num_free,
                   "kv_capacity_tokens": engine.kv_capacity_tokens,
                   "consensus_round": args.consensus_round or None,
                   "consensus_reached": sum(1 for o in orchs if o.result is not None and o.result.consensus),
                   "forced_tokens": forced,
                   "engine_ms_per_round": round(sum(eng_ms.values()) / n_timed, 2),
                   "engine_prefill_ms_per_round": round(sum(pre_ms.values()) / n_timed, 2),
                   "engine_decode_ms_per_round": round(sum(dec_ms.values()) / n_timed, 2),
                   "host_ms_per_round": round(ms_round - sum(eng_ms.values()) / n_timed, 2)},
    }
    # per-rank facts every rank contributes (one gloo gather): who took part in C1, and whether
    # each rank's decode ran as captured graphs
    per_rank = cl.all_gather_object({"c1_contributions": getattr(pool, "c1_contributions", 0),
                                     "graph_replays": engine.stats.get("graph_replays", 0),
                                     "capture_fallbacks": engine.stats.get("capture_fallbacks", 0),
                                     "use_graphs": bool(engine.ecfg.use_graphs)})
    out["detail"]["c1_contributions_per_rank"] = [r["c1_contributions"] for r in per_rank]
    out["detail"]["graph_replays_per_rank"] = [r["graph_replays"] for r in per_rank]
    out["detail"]["capture_fallbacks"] = sum(r["capture_fallbacks"] for r in per_rank)
    out["detail"]["graphs_per_rank"] = [r["use_graphs"] for r in per_rank]
    out["detail"]["c1_disagreements"] = getattr(pool, "c1_disagreements", 0)
    if cl.rank == 0 and not sim and args.scaling == "strong" and T > 1 and n_tables == 1:
        out["detail"]["prediction"] = _predict(args, T, engine)
    if cl.rank == 0 and args.write_calibration and getattr(engine.tp, "oneshot", None) is not None:
        os_ = engine.tp.oneshot
        cal = {"ar_us": os_.latency_us,
               "fused_ar_saving_us": os_.fused_saving_us if os_.fused and os_.fused_saving_us else 0.0,
               "source": f"bench.py tp{T} on {N} GPU(s), K9 probe at engine creation", "measured_unix": time.time()}
        with open(args.write_calibration, "w") as f:
            json.dump(cal, f, indent=1)
    if args.c1_events:
        with open(f"{args.c1_events}.r{cl.rank}.json", "w") as f:
            json.dump({"rank": cl.rank, "events": pool.events, "ns": pool.event_ns}, f)
    if cl.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    cl.barrier()
    from theroundtaible_amd.parallel.cluster import shutdown_cluster
    shutdown_cluster()
    return 0


if __name__ == "__main__":
    sys.exit(main())
