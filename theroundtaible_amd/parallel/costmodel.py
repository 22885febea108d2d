"""Per-rank wall-clock model of a knight group's decode step and discussion round (VERDICT r2
next #5: placement by a measured model, not a fixed step target).

A decode step of a Llama-family engine on ``tp`` GPUs holding ``B`` knights costs, per rank,

    L x [ gemm(qkv) + attn + gemm(o) + gemm(gate_up) + gemm(down) + 2 x allreduce(tp) ]
      + gemm(lm_head) + gather(tp) + sampler + step overhead

with ``gemm(kind) = floor(kind) + bytes / tp / BW`` and ``attn = floor + KV bytes / tp / BW``
(the grouped K3 reads a table's shared prefix once per step). Every constant is calibrated
from MI355X measurements of THIS engine's kernels (``Calibration`` cites the profile each
comes from); only the xGMI all-reduce latency (K9 one-shot, ``ar_us``) is an estimate until
an 8-GPU node runs — tools/tp_cost.py prints the curve for a range of it.

A round (parallel mode) = the group's prefill of the new transcript + ``new_tokens`` steps;
sequential mode (reference semantics, /root/reference/src/orchestrator.ts:361-536) runs its
knights one after another at B = 1.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..models.config import ModelConfig, get_config


@dataclass
class Calibration:
    # decode GEMM: floor (launch + first round trip + epilogue) and sustained weight stream.
    # tools/microbench.py --only gemm_tp, round 4 (profiles/r04/microbench_gemm_tp_gattn.log: NORM
    # prologues, residual epilogues): o tp8 4.2 MB 3.5 us, down tp8 14.7 MB 5.1 us, gate_up tp8
    # 29 MB 9.4 us, qkv tp8 6.3 MB 6.8 us, tp2 qkv 25 MB 7.4 us; tp1 qkv 50 MB 11.2 us, gate_up
    # 235 MB 36-40 us, down 117 MB 19 us, lm_head 1.05 GB 150-176 us. A pure 16-B/lane weight stream
    # of a launch costs 2.2 us (1 workgroup) to 3.5 us (256 x 16 KB) before its bytes
    # (tools/probes/stream_probe.hip, profiles/r04/stream_probe.csv)
    hbm_tbps: float = 6.0
    gemm_floor_us: Dict[str, float] = field(default_factory=lambda: {
        "qkv": 5.7, "o": 2.8, "gate_up": 4.6, "down": 2.7, "lm_head": 2.5})
    # grouped decode attention: floor + K/V stream (profiles/r02_bench_kernels_final_s5.md: 25.9 us
    # per layer at ~40K shared keys, tp1; r03 split cap for small KV-head shards)
    attn_floor_us: float = 8.0
    attn_tbps: float = 6.3
    # K9 one-shot all-reduce per call: 5.4 us between 2 ranks' IPC buffers on ONE GPU
    # (tools/oneshot_check.py --bench, r03); the xGMI hop is an ESTIMATE (no 8-GPU node yet)
    ar_us: float = 8.0
    # vocab-parallel logits gather per step: K9's one-shot all-gather, 9.4-9.6 us for [3, 16032] ->
    # [3, 32064] between 2 ranks sharing one GPU (profiles/r03/k9_fused_gather_shared_gpu.md); RCCL's
    # ring all-gather + permute is the fallback the creation probe compares it with
    gather_us: float = 9.5
    # the fused row-parallel GEMM + all-reduce (EPI_AR) removes the K9 launch; its saving per call is
    # measured by the creation probe on the node (bench detail k9_fused_saving_us), 0 until then
    fused_ar_saving_us: float = 0.0
    sampler_us: float = 26.0        # K6 + step bookkeeping, ONE launch (profiles/r03/bench_final_kernels_25rounds.md)
    step_overhead_us: float = 5.0   # graph-replay gaps per step (the bookkeeping is inside K6)
    # prefill: effective GEMM + attention throughput of the chunked varlen prefill (r02: 52.6 ms
    # per round for ~1.9K new tokens x 3 knights on Llama-3-8B -> ~0.6 PFLOP/s incl. attention)
    prefill_tflops: float = 600.0
    prefill_ar_gbps: float = 120.0  # RCCL ring all-reduce bus bandwidth per link (estimate)


CALIBRATION_ENV = "ROUNDTABLE_CALIBRATION"
_CAL_CACHE: Dict[str, tuple] = {}


def default_calibration() -> Calibration:
    """The calibration the model uses when none is passed: the built-in constants, overridden
    field by field by the JSON file ``$ROUNDTABLE_CALIBRATION`` names — e.g. the one
    ``bench.py --write-calibration`` writes after an N-GPU run, which carries the node's own
    measured K9 latency and fused-form saving (the xGMI numbers a 1-GPU box cannot measure), so
    ``init --placement auto`` plans with measured, not assumed, collective costs."""
    import json
    import os
    path = os.environ.get(CALIBRATION_ENV, "")
    if not path or not os.path.exists(path):
        return Calibration()
    mt = os.path.getmtime(path)
    hit = _CAL_CACHE.get(path)
    if hit is not None and hit[0] == mt:
        return hit[1]
    with open(path) as f:
        data = json.load(f)
    cal = Calibration()
    for k, v in data.items():
        if k in cal.__dataclass_fields__ and isinstance(v, (int, float)) and not isinstance(v, bool):
            setattr(cal, k, float(v))
    _CAL_CACHE[path] = (mt, cal)
    return cal


def _attn_kv_bytes(cfg: ModelConfig, tp: int, ctx_shared: int, ctx_private: int, B: int) -> float:
    kv_heads = max(1, cfg.n_kv_heads // tp)
    per_tok = kv_heads * cfg.head_dim * 2 * 2          # K and V, bf16, one layer
    return per_tok * (ctx_shared + B * ctx_private)


def decode_step_us(cfg: ModelConfig, tp: int, B: int, ctx_shared: int, ctx_private: int = 0,
                   cal: Optional[Calibration] = None) -> Tuple[float, Dict[str, float]]:
    """Predicted µs of one decode step (one token for each of the B knights) per rank."""
    cal = cal or default_calibration()
    H, D = cfg.hidden, cfg.head_dim
    hq, hkv, F = cfg.n_heads // tp, max(1, cfg.n_kv_heads // tp), cfg.ffn // tp
    bw = cal.hbm_tbps * 1e6          # bytes per µs
    shapes = {"qkv": (hq + 2 * hkv) * D * H * 2, "o": H * hq * D * 2, "gate_up": 2 * F * H * 2,
              "down": H * F * 2}
    per_layer = {k: cal.gemm_floor_us[k] + b / bw for k, b in shapes.items()}
    attn = cal.attn_floor_us + _attn_kv_bytes(cfg, tp, ctx_shared, ctx_private, B) / (cal.attn_tbps * 1e6)
    ar = 2 * max(0.0, cal.ar_us - cal.fused_ar_saving_us) if tp > 1 else 0.0
    L = cfg.n_layers
    lm = cal.gemm_floor_us["lm_head"] + (-(-cfg.vocab // tp)) * H * 2 / bw
    br = {"gemm": L * sum(per_layer.values()) + lm, "attention": L * attn, "allreduce": L * ar,
          "gather": cal.gather_us if tp > 1 else 0.0, "sampler": cal.sampler_us, "overhead": cal.step_overhead_us}
    return sum(br.values()), br


def prefill_ms(cfg: ModelConfig, tp: int, tokens: int, ctx: int, cal: Optional[Calibration] = None) -> float:
    """Chunked prefill of ``tokens`` new tokens after ``ctx`` resident ones, per rank."""
    cal = cal or default_calibration()
    if tokens <= 0:
        return 0.0
    n = cfg.n_params() - cfg.vocab * cfg.hidden        # the embedding is a gather
    flops = 2 * n * tokens + 4 * cfg.n_layers * cfg.n_heads * cfg.head_dim * tokens * (ctx + tokens / 2)
    t = flops / tp / (cal.prefill_tflops * 1e12) * 1e3
    if tp > 1:   # 2 ring all-reduces of [tokens, hidden] bf16 per layer
        msg = tokens * cfg.hidden * 2
        t += 2 * cfg.n_layers * (2 * (tp - 1) / tp * msg / (cal.prefill_ar_gbps * 1e9) * 1e3 + 0.02)
    return t


@dataclass
class RoundEstimate:
    tp: int
    knights: int
    step_us: float
    round_ms: float
    breakdown: Dict[str, float]


def round_estimate(model: str, tp: int, knights: int, new_tokens: int = 512, prefill_tokens: int = 2000,
                   ctx: int = 20000, round_mode: str = "parallel", overrides: Optional[dict] = None,
                   cal: Optional[Calibration] = None) -> RoundEstimate:
    """One group of ``knights`` same-model knights on one tp-``tp`` engine: wall-clock of one
    discussion round. ``ctx``: resident shared context per knight (the table's transcript);
    ``prefill_tokens``: new tokens per round per knight."""
    cfg = get_config(model, **(overrides or {}))
    if round_mode == "sequential":
        s, br = decode_step_us(cfg, tp, 1, ctx, 0, cal)
        r = knights * (new_tokens * s / 1e3 + prefill_ms(cfg, tp, prefill_tokens, ctx, cal))
    else:
        s, br = decode_step_us(cfg, tp, knights, ctx, prefill_tokens, cal)
        r = new_tokens * s / 1e3 + prefill_ms(cfg, tp, prefill_tokens * knights, ctx, cal)
    return RoundEstimate(tp, knights, s, r, br)


def tp_candidates(cfg: ModelConfig, n_gpus: int) -> List[int]:
    """Tensor-parallel degrees the model's shapes allow on ``n_gpus`` (KV heads split or replicated)."""
    out = []
    t = 1
    while t <= n_gpus:
        if cfg.n_heads % t == 0 and cfg.ffn % t == 0 and (cfg.n_kv_heads % t == 0 or t % cfg.n_kv_heads == 0):
            out.append(t)
        t *= 2
    return out


def best_tp(model: str, knights: int, n_gpus: int, fits=None, **kw) -> RoundEstimate:
    """The tp (<= n_gpus, allowed by the shapes and by ``fits(tp)`` memory) with the shortest
    predicted round; ties go to the smaller tp (fewer GPUs, fewer collectives)."""
    cfg = get_config(model, **(kw.get("overrides") or {}))
    best = None
    for t in tp_candidates(cfg, n_gpus):
        if fits is not None and not fits(t):
            continue
        e = round_estimate(model, t, knights, **kw)
        if best is None or e.round_ms < best.round_ms * 0.98:
            best = e
    if best is None:
        raise ValueError(f"{model}: no tensor-parallel degree <= {n_gpus} fits")
    return best


def split_plans(model: str, knights: int, n_gpus: int, fits=None, **kw) -> List[Tuple[float, List[Tuple[int, int]]]]:
    """Ways to seat ``knights`` same-model knights on ``n_gpus``: g equal groups (one engine each,
    batched decode) x tp per group, g * tp <= n_gpus. Returns (predicted round ms = slowest group,
    [(knights, tp)] per group), fastest first."""
    cfg = get_config(model, **(kw.get("overrides") or {}))
    out = []
    for g in range(1, knights + 1):
        sizes = [knights // g + (1 if i < knights % g else 0) for i in range(g)]
        for t in tp_candidates(cfg, n_gpus):
            if g * t > n_gpus or (fits is not None and not fits(t)):
                continue
            ms = max(round_estimate(model, t, k, **kw).round_ms for k in sizes)
            if kw.get("round_mode") == "sequential":   # speakers one after another: groups add up
                ms = sum(round_estimate(model, t, k, **kw).round_ms for k in sizes)
            out.append((ms, [(k, t) for k in sizes]))
    out.sort(key=lambda x: (x[0], sum(t for _, t in x[1])))
    return out


# bench.py --simulate-tp N records of the driver configuration (copies of profiles/r03/sim*.json,
# the tools/tp_cost.py inputs), shipped with the package: bench.py reads them on the GPU box
SIM_DIR = __import__("os").path.join(__import__("os").path.dirname(__file__), "calib")


def load_simulated(n: int, round_mode: str = "parallel") -> Optional[dict]:
    """The ``bench.py --simulate-tp n`` record (``sim{n}.json``; n = 1 is the plain 1-GPU run;
    sequential rounds: ``sim{n}_seq.json``)."""
    import json
    import os
    path = os.path.join(SIM_DIR, f"sim{n}.json" if round_mode == "parallel" else f"sim{n}_seq.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def strong_round_ms(sim: dict, n: int, k9_us: float, gather_us: float, fused_saving_us: float = 0.0,
                    cal: Optional[Calibration] = None) -> float:
    """Predicted ms per round of the strong-scaling bench on n GPUs: the simulated rank-0 compute
    of that tp (collectives elided) + per decode step 2L effective all-reduces (K9 latency minus
    the fused form's saving) and one logits gather + the prefill ring all-reduces."""
    cal = cal or default_calibration()
    cfg = get_config(sim["config"]["model"].split(" ")[0])
    # decode steps per round: one batched decode (parallel rounds), or one per speaker (sequential:
    # reference semantics, /root/reference/src/orchestrator.ts:361-536, every step at B = 1)
    turns = sim["config"]["knights_per_table"] if sim["config"].get("round_mode") == "sequential" else 1
    steps = sim["config"]["new_tokens_per_turn"] * turns
    comp = sim["ms_per_round"]
    if n == 1:
        return comp
    ar = max(0.0, k9_us - fused_saving_us)
    decode_comm = steps * (2 * cfg.n_layers * ar + gather_us) / 1e3
    pre_tok = sim["detail"]["prefill_tokens"] / max(1, sim["steps"]) / turns
    msg = pre_tok * cfg.hidden * 2
    prefill_ar = turns * 2 * cfg.n_layers * (2 * (n - 1) / n * msg / (cal.prefill_ar_gbps * 1e9) * 1e3 + 0.02)
    return comp + decode_comm + prefill_ar
