"""GPU scouting and knight placement for ``roundtable init`` (reference seam:
`src/commands/init.ts:255` scouts every seat in parallel, `:96-113` tool detection, `:361-373`
local seats). The MI355X equivalent scouts GPUs instead of CLIs:

* :func:`scout_gpus` runs in a CHILD process (``python -m theroundtaible_amd.parallel.placement``)
  so the CLI process itself never initializes HIP: per GPU the name / gfx arch, HBM total and
  free, CU count; plus the link matrix between GPUs from ``rocm-smi --showtopotype`` (XGMI on an
  MI355X node: every pair one hop, 7 links x ~153 GB/s per GPU).
* :func:`plan_placement` seats the knights on GPU groups. Policy ``mode``:
  - ``auto`` (default): a measured wall-clock model (parallel/costmodel.py:
    per-kernel floors + weight / KV streams calibrated on MI355X, K9 all-reduce latency per
    layer, prefill FLOPs) predicts each candidate's round time — same-model knights batched on
    one tp-N engine, or split into equal groups, for every tp the shapes and memory allow — and
    the GPUs go where the slowest group gains most (several models: the bottleneck model gets
    the next GPUs). A lone 3-knight Llama-3-8B table on 8 GPUs gets tp > 1;
  - ``spread``: one knight per GPU group (BASELINE configs 2/3/5 wording: "one knight per
    MI355X", "one-per-GPU", "TP=4 each"): tp = the largest allowed power of two with
    knights x tp <= GPUs;
  - ``pack``: round-1 policy — memory fit, then tp doubles while weights/tp streamed at
    ``hbm_tbps`` exceed ``step_ms_target``; same-model knights together.
  Memory fit everywhere: weights/tp + a KV reserve (``kv_reserve_frac`` of HBM, at least room
  for every knight of the group at ``ctx_tokens``) must fit ``usable_frac`` of HBM; tp must
  split the query heads and FFN, and split or replicate the KV heads.
"""
from __future__ import annotations

import json
import math
import os
import re
import subprocess
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

GIB = 1 << 30


@dataclass
class GpuInfo:
    index: int
    name: str = ""
    arch: str = ""
    hbm_bytes: int = 0
    free_bytes: int = 0
    cus: int = 0


@dataclass
class Inventory:
    gpus: List[GpuInfo] = field(default_factory=list)
    links: Dict[str, str] = field(default_factory=dict)    # "i-j" -> "XGMI" | "PCIE" | ...

    def link(self, i: int, j: int) -> str:
        return self.links.get(f"{min(i, j)}-{max(i, j)}", "unknown")

    def to_json(self) -> dict:
        return {"gpus": [g.__dict__ for g in self.gpus], "links": self.links}

    @classmethod
    def from_json(cls, d: dict) -> "Inventory":
        return cls([GpuInfo(**g) for g in d.get("gpus", [])], dict(d.get("links", {})))


def _probe_in_child() -> dict:
    """Runs inside the child process: torch device properties + rocm-smi link types."""
    out = {"gpus": [], "links": {}}
    try:
        import torch
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            free, total = torch.cuda.mem_get_info(i)
            out["gpus"].append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", ""),
                                "hbm_bytes": int(total), "free_bytes": int(free),
                                "cus": int(p.multi_processor_count)})
    except Exception:  # noqa: BLE001 - no GPU / no torch: empty inventory
        pass
    out["links"] = _rocm_smi_links()
    return out


def _rocm_smi_links() -> Dict[str, str]:
    exe = "/opt/rocm/bin/rocm-smi"
    if not os.path.exists(exe):
        return {}
    try:
        r = subprocess.run([exe, "--showtopotype", "--json"], capture_output=True, text=True, timeout=20)
        return parse_topotype(r.stdout)
    except (OSError, subprocess.SubprocessError):
        return {}


def parse_topotype(text: str) -> Dict[str, str]:
    """rocm-smi ``--showtopotype --json``: ``"(Topology) Link type between DRM devices 0 and 1": "XGMI"``."""
    try:
        data = json.loads(text)
    except (ValueError, TypeError):
        return {}
    links: Dict[str, str] = {}

    def walk(o):
        if isinstance(o, dict):
            for k, v in o.items():
                m = re.search(r"between DRM devices (\d+) and (\d+)", str(k))
                if m and isinstance(v, str):
                    i, j = int(m.group(1)), int(m.group(2))
                    if i != j:
                        links[f"{min(i, j)}-{max(i, j)}"] = v.strip().upper()
                else:
                    walk(v)
    walk(data)
    return links


def scout_gpus(timeout_s: float = 120.0) -> Inventory:
    """GPU inventory from a child process (the caller never initializes HIP)."""
    try:
        r = subprocess.run([sys.executable, "-m", "theroundtaible_amd.parallel.placement", "--probe"],
                           capture_output=True, text=True, timeout=timeout_s,
                           env=dict(os.environ, PYTHONPATH=os.pathsep.join(
                               [os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))]
                               + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])))
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        return Inventory.from_json(json.loads(line[-1])) if line else Inventory()
    except (OSError, subprocess.SubprocessError, ValueError):
        return Inventory()


# ---- planning -------------------------------------------------------------------------------------
def model_bytes(model: str, overrides: Optional[dict] = None) -> int:
    """bf16 weight bytes of a preset (embedding + lm_head + layers)."""
    from ..models.config import get_config
    c = get_config(model, **(overrides or {}))
    if c.arch == "gpt2":
        per_layer = 4 * c.hidden * c.hidden + 2 * c.hidden * c.ffn
        n = c.n_layers * per_layer + c.vocab * c.hidden + c.max_pos * c.hidden
    else:
        qkv = (c.n_heads + 2 * c.n_kv_heads) * c.head_dim * c.hidden
        per_layer = qkv + c.n_heads * c.head_dim * c.hidden + 3 * c.hidden * c.ffn
        n = c.n_layers * per_layer + 2 * c.vocab * c.hidden
    return 2 * n


def kv_bytes_per_token(model: str, overrides: Optional[dict] = None) -> int:
    from ..models.config import get_config
    c = get_config(model, **(overrides or {}))
    return 2 * c.n_layers * c.n_kv_heads * c.head_dim * 2


@dataclass
class PlacementPolicy:
    usable_frac: float = 0.9        # of HBM for weights + KV (activations, graphs, RCCL buffers: the rest)
    kv_reserve_frac: float = 0.3    # KV headroom kept per GPU group beyond the weights
    ctx_tokens: int = 65536         # per-knight context the KV reserve must hold at least
    hbm_tbps: float = 6.0           # sustained weight-stream bandwidth (measured 5.8-6.8 TB/s)
    step_ms_target: float = 8.0     # pack mode: decode step (weights streamed once) target
    mode: str = "auto"              # auto (cost model) | spread (one knight per group) | pack
    round_mode: str = "parallel"    # the discussion's round mode (sequential = reference semantics)
    new_tokens: int = 512           # cost model workload: decode tokens per knight turn
    prefill_tokens: int = 2000      # new prompt tokens per knight turn
    round_ctx: int = 20000          # resident transcript per knight


@dataclass
class GroupPlan:
    model: str
    tp: int
    gpus: List[int]
    knights: List[str]
    weight_gib_per_gpu: float
    step_ms: float
    reason: str
    round_ms: float = 0.0            # cost model prediction (auto / spread)


def _tp_ok(model: str, overrides: Optional[dict], tp: int) -> bool:
    from ..models.config import get_config
    c = get_config(model, **(overrides or {}))
    return ((c.n_kv_heads % tp == 0 or tp % c.n_kv_heads == 0) and c.n_heads % tp == 0 and c.ffn % tp == 0)


def _fits(pol: PlacementPolicy, hbm: int, model: str, ov: Optional[dict], knights: int, tp: int) -> bool:
    w, kvtok = model_bytes(model, ov), kv_bytes_per_token(model, ov)
    return w / tp + max(pol.kv_reserve_frac * hbm, knights * pol.ctx_tokens * kvtok / tp) <= pol.usable_frac * hbm


def plan_placement(knights: Sequence[dict], inv: Inventory, policy: Optional[PlacementPolicy] = None) -> List[GroupPlan]:
    """``knights``: [{"name", "model", "overrides"?}] in seat order. Returns GroupPlans (one engine
    each: its knights batch into one decode on its GPU group); every knight appears in exactly
    one plan."""
    pol = policy or PlacementPolicy()
    if pol.mode in ("auto", "spread") and inv.gpus:
        plans = _plan_modelled(knights, inv, pol)
        if plans is not None:
            return plans
    return _plan_pack(knights, inv, pol)


def _plan_modelled(knights: Sequence[dict], inv: Inventory, pol: PlacementPolicy) -> Optional[List[GroupPlan]]:
    """auto / spread placement from the cost model; None when the models cannot each get their
    own GPUs (more models than GPUs: the pack policy shares GPUs between engines)."""
    from .costmodel import round_estimate, tp_candidates
    from ..models.config import get_config
    n = len(inv.gpus)
    hbm = min(g.hbm_bytes for g in inv.gpus) or 288 * GIB
    by_model: Dict[str, List[dict]] = {}
    for k in knights:
        by_model.setdefault(k["model"], []).append(k)
    kw = dict(new_tokens=pol.new_tokens, prefill_tokens=pol.prefill_tokens, ctx=pol.round_ctx,
              round_mode=pol.round_mode)

    def groups_ms(m: str, layout: List[tuple]) -> float:
        ov = by_model[m][0].get("overrides")
        per = [round_estimate(m, t, k, overrides=ov, **kw).round_ms for k, t in layout]
        return sum(per) if pol.round_mode == "sequential" else max(per)

    def options(m: str, budget: int) -> List[tuple]:
        """(ms, layout) of every equal split of the model's knights into g groups x tp <= budget."""
        ov = by_model[m][0].get("overrides")
        cfg = get_config(m, **(ov or {}))
        nk = len(by_model[m])
        out = []
        gs = [nk] if pol.mode == "spread" else range(1, nk + 1)
        for g in gs:
            sizes = [nk // g + (1 if i < nk % g else 0) for i in range(g)]
            for t in tp_candidates(cfg, budget):
                if g * t <= budget and all(_fits(pol, hbm, m, ov, s_, t) for s_ in sizes):
                    layout = [(s_, t) for s_ in sizes]
                    out.append((groups_ms(m, layout), layout))
        if pol.mode == "spread" and out:       # one knight per group: the widest tp that fits
            out = [max(out, key=lambda o: (o[1][0][1], -o[0]))]
        out.sort(key=lambda o: (o[0], sum(t for _, t in o[1])))
        return out

    order = sorted(by_model, key=lambda m: -model_bytes(m, by_model[m][0].get("overrides")))
    # 1. every model at its cheapest-in-GPUs feasible layout
    state: Dict[str, tuple] = {}
    for m in order:
        opts = options(m, n)
        if not opts:
            return None
        state[m] = min(opts, key=lambda o: (sum(t for _, t in o[1]), o[0]))
    if sum(sum(t for _, t in state[m][1]) for m in order) > n:
        return None
    # 2. GPUs to the bottleneck model while its predicted round shrinks
    while True:
        used = sum(sum(t for _, t in state[m][1]) for m in order)
        m = max(order, key=lambda x: state[x][0])
        mine = sum(t for _, t in state[m][1])
        better = [o for o in options(m, n - used + mine) if o[0] < state[m][0] * 0.98]
        if not better:
            break
        state[m] = better[0]
    plans: List[GroupPlan] = []
    nxt = 0
    for m in order:
        ov = by_model[m][0].get("overrides")
        names = [k["name"] for k in by_model[m]]
        ms, layout = state[m]
        w = model_bytes(m, ov)
        for k, t in layout:
            est = round_estimate(m, t, k, overrides=ov, **kw)
            why = (f"cost model: {est.round_ms:.0f} ms/round predicted ({pol.round_mode})" if pol.mode == "auto"
                   else f"one knight per group, widest tp ({est.round_ms:.0f} ms/round predicted)")
            plans.append(GroupPlan(m, t, list(range(nxt, nxt + t)), names[:k], round(w / t / GIB, 1),
                                   round(est.step_us / 1e3, 2), why, round(est.round_ms, 1)))
            names = names[k:]
            nxt += t
    return plans


def _plan_pack(knights: Sequence[dict], inv: Inventory, pol: PlacementPolicy) -> List[GroupPlan]:
    n = len(inv.gpus)
    by_model: Dict[str, List[dict]] = {}
    for k in knights:
        by_model.setdefault(k["model"], []).append(k)
    if n == 0:
        return [GroupPlan(m, 1, [], [k["name"] for k in ks], round(model_bytes(m, ks[0].get("overrides")) / GIB, 1),
                          0.0, "no GPU visible: CPU") for m, ks in by_model.items()]
    hbm = min(g.hbm_bytes for g in inv.gpus) or 288 * GIB

    def step_ms(w, tp):
        return w / tp / (pol.hbm_tbps * 1e12) * 1e3

    # 1. per model: smallest tp that fits (weights + KV reserve), biggest models first
    order = sorted(by_model, key=lambda m: -model_bytes(m, by_model[m][0].get("overrides")))
    tps: Dict[str, int] = {}
    why: Dict[str, str] = {}
    for m in order:
        ov = by_model[m][0].get("overrides")
        w, kvtok, nk = model_bytes(m, ov), kv_bytes_per_token(m, ov), len(by_model[m])
        tp = 1
        while tp < n and (w / tp + max(pol.kv_reserve_frac * hbm, nk * pol.ctx_tokens * kvtok / tp)
                          > pol.usable_frac * hbm or not _tp_ok(m, ov, tp)):
            tp *= 2
        tps[m], why[m] = min(tp, n), ("fits one GPU" if tp == 1 else "memory fit")
    # 2. decode-latency target while GPUs are free
    free = n - sum(tps.values())
    for m in order:
        ov = by_model[m][0].get("overrides")
        w = model_bytes(m, ov)
        while step_ms(w, tps[m]) > pol.step_ms_target and free >= tps[m] and _tp_ok(m, ov, 2 * tps[m]):
            free -= tps[m]
            tps[m] *= 2
            why[m] = f"decode step <= {pol.step_ms_target:g} ms"
    # 3. assign GPU groups in order; out of GPUs -> share (split KV pool, own HIP stream)
    plans: List[GroupPlan] = []
    nxt = 0
    for m in order:
        ov = by_model[m][0].get("overrides")
        tp, note = tps[m], why[m]
        if nxt + tp <= n:
            gpus = list(range(nxt, nxt + tp))
            nxt += tp
        else:
            start = (nxt % n) // tp * tp if tp <= n else 0
            gpus = list(range(start, min(n, start + tp)))
            nxt += tp
            note += "; shares GPUs with another model (KV pool split, own HIP stream)"
        w = model_bytes(m, ov)
        plans.append(GroupPlan(m, tp, gpus, [k["name"] for k in by_model[m]], round(w / tp / GIB, 1),
                               round(step_ms(w, tp), 2), note))
    return plans


def main() -> int:
    if "--probe" in sys.argv:
        print(json.dumps(_probe_in_child()), flush=True)
        return 0
    inv = scout_gpus()
    print(json.dumps(inv.to_json(), indent=2))
    return 0


if __name__ == "__main__":
    sys.exit(main())
