"""Knight backends for a multi-GPU (torchrun, one process per GPU) ``discuss`` / ``summon``.

Launched as ``torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m theroundtaible_amd
discuss "..."``, every rank runs the same CLI/orchestrator program (SPMD,
:mod:`theroundtaible_amd.knights.distributed`). This module turns the project config into

* a **placement**: knight -> ranks. ``adapter_config[id].engine.gpus`` names the ranks (the
  node's GPUs, one rank each); ``tp`` must equal ``len(gpus)``. Knights without ``gpus`` are
  dealt round-robin over the ranks, ``tp`` consecutive ranks at a time;
* **TP process groups**: one ``new_group`` per distinct multi-rank placement, created in the
  same order on every rank (``new_group`` is collective);
* **local engines**: only for knights placed on this rank, one engine per (model, weights,
  placement) so knights sharing a placement batch into one decode; a TP knight's engine is
  built with :class:`~theroundtaible_amd.parallel.tp.TPInfo` of its group (RCCL all-reduce
  and vocab all-gather inside its forward);
* one :class:`RemoteKnight` per adapter id, all backed by one :class:`DistributedPool`,
  whose C1 exchange returns every knight's output on every rank.
"""
from __future__ import annotations

import datetime
import threading
from typing import Dict, List, Tuple

from ..config import engine_settings
from ..engine.engine import Engine, EngineConfig
from ..engine.sampler import SamplingParams
from ..parallel.cluster import Cluster, load_group_for
from ..parallel.tp import TPInfo
from ..types import RoundtableConfig
from ..utils.local_detect import resolve_model
from ..utils import failsafe
from ..utils.ui import NULL_UI, UI
from .distributed import DistributedPool, RemoteKnight
from .engine_backend import EngineBackend
from .registry import display_name
from .script import ConsensusScript


def plan_placement(config: RoundtableConfig, world: int) -> Dict[str, List[int]]:
    """adapter id -> ranks (first = leader). Deterministic: every rank computes the same plan."""
    placement: Dict[str, List[int]] = {}
    nxt = 0
    for k in config.knights:
        aid = k.adapter
        if aid in placement:
            continue
        st = engine_settings(config, aid)
        tp = int(st.get("tp", 1) or 1)
        gpus = st.get("gpus")
        if isinstance(gpus, list) and gpus:
            ranks = [int(g) for g in gpus]
            if len(ranks) != tp and tp != 1:
                raise ValueError(f"{aid}: engine.tp={tp} but engine.gpus has {len(ranks)} entries")
        else:
            ranks = [(nxt + t) % world for t in range(tp)]
            nxt = (nxt + tp) % world
        bad = [r for r in ranks if r < 0 or r >= world]
        if bad:
            raise ValueError(f"{aid}: engine.gpus {ranks} outside the {world} launched ranks")
        placement[aid] = ranks
    return placement


def build_spmd_backends(config: RoundtableConfig, cluster: Cluster, ui: UI = NULL_UI,
                        max_new_tokens: int = None) -> Tuple[Dict[str, RemoteKnight], DistributedPool]:
    import torch.distributed as dist
    placement = plan_placement(config, cluster.world)
    groups: Dict[Tuple[int, ...], object] = {}
    load_groups: Dict[Tuple[int, ...], object] = {}
    for ranks in placement.values():           # identical order on every rank (collective)
        key = tuple(ranks)
        if len(key) > 1 and key not in groups:
            # the containment timeout (torch's new_group default would be 30 min); safe for the
            # group's first collective because Engine meets on the load group before it
            groups[key] = dist.new_group(list(key), timeout=datetime.timedelta(seconds=cluster.timeout_s)) \
                if cluster.distributed else None
            load_groups[key] = load_group_for(key) if cluster.distributed else None
    engines: Dict[tuple, Tuple[Engine, threading.Lock]] = {}
    local: Dict[str, EngineBackend] = {}
    tokenizer = None
    for k in config.knights:
        aid = k.adapter
        ranks = placement[aid]
        if cluster.rank not in ranks or aid in local:
            continue
        st = engine_settings(config, aid)
        tp = TPInfo(size=len(ranks), rank=ranks.index(cluster.rank), group=groups.get(tuple(ranks)),
                    load_group=load_groups.get(tuple(ranks)))
        ekey = (st["model"], str(st.get("weights", "random:0")), str(st.get("dtype", "bf16")), tuple(ranks))
        if ekey not in engines:
            model, overrides = resolve_model(st["model"], str(st.get("weights", "random:0")), st.get("model_overrides"))
            dev = "cpu" if str(st.get("device", "")) == "cpu" else cluster.device
            ecfg = EngineConfig(model=model, weights=str(st.get("weights", "random:0")),
                                dtype=str(st.get("dtype", "bf16")), device=dev,
                                block_size=int(st.get("kv_block_size", 32)),
                                kv_cache_fraction=float(st.get("kv_cache_fraction", 0.85)),
                                max_kv_tokens=st.get("max_kv_tokens"),
                                use_graphs=bool(st.get("use_graphs", True)) and dev.startswith("cuda"),
                                model_overrides=overrides)
            if not ecfg.device.startswith("cuda"):
                ecfg.dtype = "fp32"
            with failsafe.stage("engine_load"):
                engines[ekey] = (Engine(ecfg, tp), threading.Lock())
        engine, lock = engines[ekey]
        tokenizer = tokenizer or engine.tokenizer
        params = SamplingParams(temperature=float(st.get("temperature", 0.7)), top_p=float(st.get("top_p", 0.95)),
                                top_k=int(st.get("top_k", 0)), seed=int(st.get("seed", 0)),
                                max_new_tokens=int(max_new_tokens or st.get("max_new_tokens", 512)),
                                ignore_eos=bool(st.get("ignore_eos", False)),
                                stop_on_consensus=bool(st.get("stop_on_consensus", True)))
        local[aid] = EngineBackend(display_name(aid, config), aid, engine, params, lock,
                                   script=ConsensusScript.from_config(st.get("scripted_consensus")))
        ui.ok(f"  ✓ {k.name}: {st['model']} on rank(s) {ranks}" + (f" (tp={len(ranks)})" if len(ranks) > 1 else ""))
    # no rank enters a turn-time (short-timeout) collective before every rank has loaded its
    # engines: ranks load one engine after another, a real checkpoint can take minutes longer on
    # one of them; the wait runs under the load limit
    with failsafe.stage("engine_load"):
        cluster.load_rendezvous()
    if tokenizer is None:   # a rank hosting no knight still decodes exchanged ids
        from ..engine.tokenizer import get_tokenizer
        from ..models.config import get_config
        st = engine_settings(config, config.knights[0].adapter)
        model, overrides = resolve_model(st["model"], str(st.get("weights", "random:0")), st.get("model_overrides"))
        tokenizer = get_tokenizer(get_config(model, **overrides).vocab, str(st.get("weights", "random:0")))
    # every tensor-parallel group agrees at each turn start that all its ranks arrived (within the
    # turn timeout) before entering its collectives: a stalled rank skips the knight's turn on
    # every rank instead of hanging the table
    pool = DistributedPool(cluster, placement, local, tokenizer, turn_rendezvous=True)
    backends = {aid: RemoteKnight(pool, aid, display_name(aid, config), aid) for aid in placement}
    return backends, pool
