"""SPMD knight pool: every rank runs the same orchestrator; knights run where they are placed.

All ranks execute the identical host program (same config, same broadcast shuffle
seed), so they build identical prompts and reach identical consensus decisions.
For each batch of turns the pool

1. runs the knights placed on this rank on the local engine (one batched decode; for a
   TP knight all ranks of its group run it in lockstep — RCCL all-reduce inside);
2. exchanges the results (C1, :mod:`theroundtaible_amd.parallel.exchange`): token
   ids via an RCCL all-gather, metadata via the gloo control group;
3. returns every knight's result on every rank.

Sequential (reference) round mode calls this with one turn at a time: only the
speaker's group computes while the others wait in the collective.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence, Tuple, Union  # noqa: F401

from ..errors import AdapterError
from ..parallel.cluster import Cluster
from ..parallel.exchange import TokenExchange, exchange_token_ids
from ..utils import failsafe, trace
from .base import KnightBackend, TurnRequest, TurnResult


class DistributedPool:
    def __init__(self, cluster: Cluster, placement: Dict[str, List[int]], local: Dict[str, KnightBackend],
                 tokenizer=None, max_reply_tokens: int = 4096, turn_rendezvous: bool = False):
        """``placement``: knight name -> ranks hosting it (first = leader). ``local``: name -> backend here.
        ``max_reply_tokens``: width of the static C1 buffers (longer replies take the shape-agreeing path).
        ``turn_rendezvous``: every tensor-parallel group agrees, through the launcher's key-value store
        and within the turn timeout, that ALL its ranks reached a turn before any of them enters its
        collectives (``roundtable discuss`` & co.; see :meth:`_rendezvous`)."""
        self.cluster = cluster
        self.placement = placement
        self.local = local
        self.tokenizer = tokenizer
        self.turn_rendezvous = turn_rendezvous and cluster.distributed
        self._rv_count: Dict[tuple, int] = {}
        self._calls = 0
        self.rendezvous_skips = 0
        self.exchange_ms: List[float] = []
        self.exchange: Optional[TokenExchange] = None
        self.events: List[str] = []     # C1 ordering record (c1_start / speculate / c1_wait)
        self.event_ns: List[int] = []   # CLOCK_MONOTONIC ns of each event (the kernel-trace clock)
        self.speculate = os.environ.get("ROUNDTABLE_C1_SPECULATE", "1") != "0"
        if cluster.distributed:
            led = [sum(1 for r in placement.values() if r[0] == k) for k in range(cluster.world)]
            self.exchange = TokenExchange(cluster, max(led), max_reply_tokens, cluster.device)
        budgets = [b.max_source_chars() for b in local.values()]
        mine = min([b for b in budgets if b is not None], default=200_000)
        self._src_budget = int(-cluster.max_scalar(-float(mine))) if cluster.distributed else mine

    def leader(self, name: str) -> int:
        return self.placement[name][0]

    def _speculate(self, pairs, local_res, mine_idx) -> None:
        """C1 overlap: while the remote replies are in flight, ask each table's predictor
        (``TurnRequest.speculate``, set by the orchestrator) for its next prompt as far as THIS
        rank's finished turns determine it, and prefill that prefix on every local engine hosting
        one of the table's knights (``KnightBackend.prefetch`` -> ``Engine.warm_shared``). The
        next turn keeps the prefilled KV by LCP; a wrong guess costs only the prefill.
        ROUNDTABLE_C1_SPECULATE=0 disables it."""
        if not self.speculate:
            return
        local_ok = {pairs[i][1].seq_key: local_res[i] for i in mine_idx
                    if i in local_res and not isinstance(local_res[i], BaseException)}
        preds: Dict[int, tuple] = {}
        for i in mine_idx:
            f = getattr(pairs[i][1], "speculate", None)
            if f is not None:
                preds.setdefault(id(f), (f, []))[1].append(i)
        for f, idxs in preds.values():
            try:
                prompt = f(local_ok)
            except Exception:  # noqa: BLE001 - a failed guess only loses the overlap
                prompt = None
            if prompt is None:
                continue
            self._event("speculate")
            done = set()
            for i in idxs:
                b = self.local[pairs[i][0].knight_name]
                if b.group_key() in done:
                    continue
                done.add(b.group_key())
                with trace.range("C1 overlap: speculative prefill"):
                    try:
                        b.prefetch(pairs[i][1].seq_key, prompt)
                    except Exception:  # noqa: BLE001 - a failed speculation only loses the overlap;
                        pass           # a real device fault surfaces in the next turn
            self._event("speculate_end")

    def _event(self, name: str) -> None:
        self.events.append(name)
        self.event_ns.append(time.monotonic_ns())
        if len(self.events) > 4096:
            del self.events[:1024], self.event_ns[:1024]

    def _store(self):
        """A key-value store every rank of the launch shares, opened once per pool. Under torchrun
        (the SPMD commands' launcher) that is a client of the elastic agent's TCP store at
        MASTER_ADDR:MASTER_PORT — the same store torch's env:// rendezvous joined — under a prefix of
        our own; a process group initialised any other way falls back to the default group's store
        (``_get_default_store``, private API)."""
        if getattr(self, "_kv_store", None) is None:
            import datetime
            import torch.distributed as dist
            if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true" and os.environ.get("MASTER_PORT"):
                client = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                                       is_master=False, timeout=datetime.timedelta(seconds=300))
                self._kv_store = dist.PrefixStore("roundtable/", client)
            else:
                self._kv_store = dist.distributed_c10d._get_default_store()
        return self._kv_store

    def _rendezvous(self, ranks: tuple, wait_s: float) -> bool:
        """Turn-start agreement of one tensor-parallel group, outside its process groups (the
        launcher's TCP key-value store): each rank counts itself in, and the FIRST rank to see
        either every rank arrived ("go") or its wait expire ("skip") fixes the decision with one
        compare-and-set; every rank — a late one included — takes that decision. A rank that
        stalls before a turn (a hung host call, a slow previous step) thus makes the whole group
        skip the turn with a timeout error within ``wait_s``, instead of its peers blocking inside
        the turn's first collective for the process-group timeout, and a late rank never enters
        collectives its peers have abandoned (reference: a failed turn is skipped and the round
        continues, /root/reference/src/orchestrator.ts:521-535)."""
        store = self._store()
        n = self._rv_count[ranks] = self._rv_count.get(ranks, 0) + 1
        key = f"rt/turn/{'-'.join(map(str, ranks))}/{n}"
        store.add(key + "/n", 1)
        deadline = time.monotonic() + wait_s
        while True:
            if store.check([key + "/d"]):
                dec = store.get(key + "/d")
                break
            if store.add(key + "/n", 0) >= len(ranks):
                dec = store.compare_set(key + "/d", "", "go")
                break
            if time.monotonic() > deadline:
                dec = store.compare_set(key + "/d", "", "skip")
                break
            time.sleep(0.002)
        # the last of the group's ranks to read the decision removes the turn's keys: the store
        # holds O(groups) keys for the whole session, not O(turns). A rank that never
        # reaches this turn leaves them; the decision itself is already fixed either way.
        if store.add(key + "/r", 1) >= len(ranks):
            for k in (key + "/n", key + "/d", key + "/r"):
                store.delete_key(k)
        return dec == b"go"

    def execute_round(self, pairs: Sequence[Tuple["RemoteKnight", TurnRequest]],
                      timeout_s: float) -> List[Union[TurnResult, BaseException]]:
        rank = self.cluster.rank
        self._calls += 1
        mine_idx = [i for i, (k, _) in enumerate(pairs) if rank in self.placement[k.knight_name]]
        local_res: Dict[int, Union[TurnResult, BaseException]] = {}
        # group local work by underlying backend group (one batched decode per engine)
        groups: Dict[object, List[int]] = {}
        for i in mine_idx:
            b = self.local[pairs[i][0].knight_name]
            groups.setdefault(b.group_key(), []).append(i)
        # tensor-parallel groups first, in one global order (their placements sorted), so a
        # group's k-th place bounds when its ranks can all arrive: k turns of at most timeout_s
        # each; single-rank engines after them
        tp_order = sorted({tuple(self.placement[k.knight_name]) for k, _ in pairs
                           if len(self.placement[k.knight_name]) > 1})

        def place(idxs):
            pl = tuple(self.placement[pairs[idxs[0]][0].knight_name])
            return tp_order.index(pl) if pl in tp_order else len(tp_order)

        budget = (len(tp_order) + 1) * timeout_s + 30.0
        with failsafe.stage(f"turn {self._calls}", limit_s=budget if self.turn_rendezvous else None):
            for idxs in sorted(groups.values(), key=place):
                first = self.local[pairs[idxs[0]][0].knight_name]
                ranks = tuple(self.placement[pairs[idxs[0]][0].knight_name])
                wait_s = (place(idxs) + 1) * timeout_s
                if self.turn_rendezvous and len(ranks) > 1 and not self._rendezvous(ranks, wait_s):
                    self.rendezvous_skips += 1
                    for i in idxs:
                        local_res[i] = AdapterError(pairs[i][0].name, f"a rank of its tensor-parallel group {list(ranks)} "
                                                    f"did not reach the turn within {wait_s:.0f} s; turn skipped "
                                                    "on every rank of the group", kind="timeout")
                    continue
                outs = first.execute_group([(self.local[pairs[i][0].knight_name], pairs[i][1]) for i in idxs],
                                           timeout_s)
                for i, o in zip(idxs, outs):
                    local_res[i] = o
        if len(mine_idx) == len(pairs) and all(len(self.placement[k.knight_name]) == self.cluster.world
                                               for k, _ in pairs):
            # every knight of the batch spans EVERY rank (one tensor-parallel group: the strong-
            # scaling layout): each rank already holds every result, identical across the group
            # (same sampled ids from the same gathered logits) — no token exchange is needed. The
            # ranks still agree on each turn's ok / error status (one small gloo gather): a turn
            # that failed on some ranks only (a per-rank deadline, a host-side error) takes the
            # normal C1 path below, so every rank records the leader's outcome
            status = [isinstance(local_res[i], BaseException) for i in range(len(pairs))]
            if all(s == status for s in self.cluster.all_gather_object(status)):
                self.exchange_ms.append(0.0)
                self.c1_skipped = getattr(self, "c1_skipped", 0) + 1
                return [local_res[i] for i in range(len(pairs))]
            self.c1_disagreements = getattr(self, "c1_disagreements", 0) + 1
        # contributions from the knights this rank leads
        led = [i for i in mine_idx if self.leader(pairs[i][0].knight_name) == rank]
        self.c1_contributions = getattr(self, "c1_contributions", 0) + len(led)
        t0 = time.perf_counter()
        meta = {}
        ids_contrib = []
        for i in led:
            o = local_res[i]
            if isinstance(o, BaseException):
                meta[i] = ("err", getattr(o, "kind", "unknown"), str(o))
            else:
                has_ids = o.ids is not None
                meta[i] = ("ok", None if has_ids else o.text, o.tokenizer, o.metrics)
                if has_ids:
                    ids_contrib.append((i, list(o.ids), getattr(o, "dev_ids", None)))
        with trace.range("C1 exchange"):
            ex = self.exchange
            if ex is None:
                self._speculate(pairs, local_res, mine_idx)
                all_meta = self.cluster.all_gather_object(meta)
                all_ids = exchange_token_ids(self.cluster, [c[:2] for c in ids_contrib], self.cluster.device)
            else:
                # the static-shape token all-gather (RCCL, from the device token buffers) is in
                # flight while this rank prefills what it already knows of the next prompt and
                # the gloo metadata round runs; a rank whose replies overflow the static buffers
                # says so in its metadata and every rank then joins the shape-agreeing fallback
                fits = ex.fits(ids_contrib)
                ex.start(ids_contrib if fits else [])
                self._event("c1_start")
                self._speculate(pairs, local_res, mine_idx)
                meta[-1] = not fits
                all_meta = self.cluster.all_gather_object(meta)
                all_ids = ex.wait()
                self._event("c1_wait")
                if any(m.get(-1) for m in all_meta):
                    all_ids.update(exchange_token_ids(self.cluster, [] if fits else [c[:2] for c in ids_contrib],
                                                      self.cluster.device))
        self.exchange_ms.append((time.perf_counter() - t0) * 1e3)
        merged: Dict[int, tuple] = {}
        for m in all_meta:
            merged.update({k: v for k, v in m.items() if k != -1})
        results: List[Union[TurnResult, BaseException]] = []
        for i, (k, _) in enumerate(pairs):
            m = merged.get(i)
            if m is None:
                results.append(AdapterError(k.name, "no rank hosted this knight", kind="device"))
            elif m[0] == "err":
                results.append(AdapterError(k.name, m[2], kind=m[1]))
            else:
                _, text, tok, metrics = m
                ids = all_ids.get(i)
                if text is None:
                    if i in local_res and not isinstance(local_res[i], BaseException):
                        text = local_res[i].text   # leader/local copy: exact text
                    else:
                        text = self.tokenizer.decode(ids) if self.tokenizer is not None else ""
                results.append(TurnResult(text, ids, tok, dict(metrics or {})))
        return results


class RemoteKnight(KnightBackend):
    """Orchestrator-facing backend for one knight of a :class:`DistributedPool`."""

    def __init__(self, pool: DistributedPool, knight_name: str, name: str, adapter_id: str):
        self.pool = pool
        self.knight_name = knight_name
        self.name = name
        self.adapter_id = adapter_id

    def group_key(self):
        return id(self.pool)

    def max_source_chars(self) -> Optional[int]:
        return self.pool._src_budget

    def execute_group(self, pairs, timeout_s):
        return self.pool.execute_round(pairs, timeout_s)

    def execute_many(self, reqs, timeout_s):
        return self.pool.execute_round([(self, r) for r in reqs], timeout_s)
