"""GPU scouting and knight placement for ``roundtable init`` (reference seam:
`src/commands/init.ts:255` scouts every seat in parallel, `:96-113` tool detection, `:361-373`
local seats). The MI355X equivalent scouts GPUs instead of CLIs:

* :func:`scout_gpus` runs in a CHILD process (``python -m theroundtaible_amd.parallel.placement``)
  so the CLI process itself never initializes HIP: per GPU the name / gfx arch, HBM total and
  free, CU count; plus the link matrix between GPUs from ``rocm-smi --showtopotype`` (XGMI on an
  MI355X node: every pair one hop, 7 links x ~153 GB/s per GPU).
* :func:`plan_placement` chooses each model's tensor-parallel degree and GPU group:
  - memory fit: weights/tp + a KV reserve (``kv_reserve_frac`` of HBM, at least room for every
    knight of the model at ``ctx_tokens``) must fit ``usable_frac`` of HBM;
  - decode latency: while GPUs are free, tp doubles until weights/tp streamed at ``hbm_tbps``
    take <= ``step_ms_target`` per token (Llama-3-70B: 141 GB / 6 TB/s = 23.5 ms at tp=1 -> tp=4,
    5.9 ms; Llama-3-8B: 2.7 ms -> tp=1); tp must divide the KV / query heads and the FFN;
  - knights of the same model are placed TOGETHER on one GPU group (one engine: batched decode
    + the ``shared`` prompt layout's single prefix KV copy);
  - different models get disjoint GPU groups while GPUs last, then share (the engines split that
    GPU's KV pool and run on their own HIP streams).
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
    step_ms_target: float = 8.0     # decode step (weights streamed once) target when GPUs allow


@dataclass
class GroupPlan:
    model: str
    tp: int
    gpus: List[int]
    knights: List[str]
    weight_gib_per_gpu: float
    step_ms: float
    reason: str


def _tp_ok(model: str, overrides: Optional[dict], tp: int) -> bool:
    from ..models.config import get_config
    c = get_config(model, **(overrides or {}))
    return ((c.n_kv_heads % tp == 0 or tp % c.n_kv_heads == 0) and c.n_heads % tp == 0 and c.ffn % tp == 0)


def plan_placement(knights: Sequence[dict], inv: Inventory, policy: Optional[PlacementPolicy] = None) -> List[GroupPlan]:
    """``knights``: [{"name", "model", "overrides"?}] in seat order. Returns one GroupPlan per model
    (its knights share one engine on one GPU group); every knight appears in exactly one plan."""
    pol = policy or PlacementPolicy()
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
