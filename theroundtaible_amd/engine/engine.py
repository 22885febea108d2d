"""The per-GPU(-group) inference engine that hosts one or more knights.

A knight turn on the engine:

1. tokenize the prompt segment-by-segment (stable prefixes; response segments keep ids);
2. longest-common-prefix match against the knight's *resident* KV sequence, roll the
   sequence back to the LCP (paged: drop tail blocks) and prefill only the delta —
   chunked, varlen-batched across all knights of this call (K4 prefill attention);
3. pre-allocate KV blocks for ``max_new_tokens`` and run the decode loop fully
   device-side: one hipGraph replay per token for the whole batch (embed -> 32 layers
   with K1/K2/K3/K5 -> lm_head -> K6 sampling -> next-input/slot/position update);
   the host only replays and, every ``sync_every / 2`` steps, copies the tokens back
   asynchronously and checks the previous copy (EOS / consensus JSON / wall clock)
   while the GPU keeps replaying;
4. detokenize; the generated ids are returned too (C1 token-id path), and the KV of
   the response stays resident for the knight's next turn.

The same class runs on CPU (reference ops, no graphs) for the GPT-2 plumbing config.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from ..consensus import parse_consensus
from ..errors import AdapterError, DeviceFlagError, EngineTimeout
from ..models.config import ModelConfig, get_config
from ..models.gpt2 import build_model
from ..models.llama import AttnMeta
from ..models.weights import materialize
from ..parallel.tp import TPInfo
from ..prompt import Prompt, PromptLike, Segment
from ..utils import failsafe, trace
from .kv_cache import KVCacheOOM, PagedKVCache, SeqState
from .sampler import SamplingParams
from .tokenizer import EngineTokenizer, get_tokenizer

# decode-graph batch buckets: exact sizes for the common knight counts (3-knight tables, 6 = two
# tables) so no padded row takes split-KV workgroups from the real ones (B=3: 240 vs 192 live)
BATCH_BUCKETS = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32)


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    weights: str = "random:0"
    dtype: str = "bf16"
    device: str = "cuda:0"
    block_size: int = 32
    num_blocks: Optional[int] = None        # None = size from free memory
    kv_cache_fraction: float = 0.85
    max_kv_tokens: Optional[int] = None     # optional cap on resident tokens
    prefill_chunk: int = 8192               # tokens per prefill forward (summed over sequences)
    prefill_key_split: bool = True          # split long prefill tiles' key ranges when tiles x KV heads < CUs / 2
    use_graphs: bool = True
    sync_every: int = 32                    # decode steps between host token readbacks
    max_batch: int = 16
    model_overrides: Dict[str, object] = field(default_factory=dict)
    # fault injection (tests / chaos runs): run_turns call index -> "raise" | "oom" |
    # "timeout" | "device". Also from ROUNDTABLE_ENGINE_FAULTS="2:oom,5:device".
    faults: Dict[int, str] = field(default_factory=dict)
    # validate paging metadata (block tables / slots in range) before every forward (ROUNDTABLE_DEBUG_CHECKS=1)
    debug_checks: bool = False
    # wrap each turn as one user message with the checkpoint's chat template (checkpoint tokenizers only)
    chat_template: bool = True
    # KV pool size in bytes (None: kv_cache_fraction of the free HBM at load); defer_kv: allocate on
    # allocate_kv() / first turn (EnginePool.finalize splits a GPU between its engines)
    kv_budget_bytes: Optional[int] = None
    defer_kv: bool = False
    # GPU weight copies: "dual" (row-major for prefill + shuffled for decode), "shuffled" (shuffled
    # only; prefill unshuffles per GEMM into scratch), "auto" = dual when 2x weights <= 35% of HBM
    weight_residency: str = "auto"


@dataclass
class Turn:
    seq_key: str
    prompt: PromptLike
    params: SamplingParams
    timeout_s: float = 1e9


@dataclass
class TurnOutput:
    text: str
    ids: List[int]
    metrics: Dict[str, float]
    error: Optional[BaseException] = None
    dev_ids: Optional[torch.Tensor] = None    # ``ids`` on the engine's device (None: host only)


def _dtype(s: str) -> torch.dtype:
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp16": torch.float16,
            "float16": torch.float16, "fp32": torch.float32, "float32": torch.float32}[s]


class Engine:
    def __init__(self, ecfg: EngineConfig, tp: Optional[TPInfo] = None):
        self.ecfg = ecfg
        self.tp = tp or TPInfo()
        self.cfg: ModelConfig = get_config(ecfg.model, **ecfg.model_overrides)
        self.device = torch.device(ecfg.device)
        self.on_gpu = self.device.type == "cuda"
        # host-staged (gloo) collectives cannot be captured in a hipGraph: graphs stay on for such a
        # group only if every in-step collective is a device-side K9 kernel (decided after K9 set-up)
        self.dtype = _dtype(ecfg.dtype)
        if not self.on_gpu and self.dtype == torch.float16:
            self.dtype = torch.float32
        # the checkpoint's own tokenizer + chat template when `weights` ships one, else the bundled BPE
        self.tokenizer: EngineTokenizer = get_tokenizer(self.cfg.vocab, ecfg.weights, ecfg.chat_template)
        t0 = time.perf_counter()
        with torch.no_grad():
            weights = materialize(self.cfg, ecfg.weights, self.device, self.dtype, self.tp)
            self.model = build_model(self.cfg, weights, self.device, self.dtype, self.tp)
            if self.on_gpu and hasattr(self.model, "decode_weights"):
                # shuffled decode copies before sizing the KV pool. Both layouts (+1x weight memory)
                # when that leaves most of HBM to KV; otherwise shuffle in place and keep ONLY the
                # shuffled weights (prefill unshuffles per GEMM): a 70B knight on one GPU keeps the
                # fused decode path and ~140 GB of KV
                wbytes = sum(t.numel() * t.element_size() for t in weights.values())
                total = torch.cuda.get_device_properties(self.device).total_memory
                mode = ecfg.weight_residency
                if mode == "auto":
                    mode = "dual" if 2 * wbytes <= 0.35 * total else "shuffled"
                del weights
                self.model.decode_weights(drop_originals=(mode == "shuffled"))
                self.weight_residency = mode
        if self.tp.size > 1 and self.tp.load_group is not None:
            # every rank of the group has its weights before the group's first collective
            import torch.distributed as dist
            with failsafe.stage("engine_load"):
                dist.barrier(group=self.tp.load_group)
        if self.on_gpu and self.tp.size > 1:
            with failsafe.stage("k9_create"):
                self.tp.setup_oneshot()      # K9: collective over the TP group; RCCL stays the fallback
            # a decode step whose every collective is a K9 kernel (all-reduce, and the one-shot
            # logits gather) can be captured even when the group's host collectives are gloo (the
            # shared-GPU rehearsal): agree on it, so every rank captures or none does
            if ecfg.use_graphs and self.tp.backend() != "nccl":
                ecfg.use_graphs = not self.tp.any_rank(not self.k9_only_step())
        if not hasattr(self, "weight_residency"):
            self.weight_residency = "dual"
        self.load_s = time.perf_counter() - t0
        # every engine issues its work on its OWN HIP stream: engines of different models sharing a
        # GPU run their batches concurrently (one host thread each, orchestrator.execute_plan)
        self.stream = torch.cuda.Stream(self.device) if self.on_gpu else None
        self._kv: Optional[PagedKVCache] = None if ecfg.defer_kv else self._alloc_kv()
        self.graphs: Dict[Tuple[int, int], "DecodeGraph"] = {}
        self._seg_cache: Dict[Tuple[str, str], List[int]] = {}
        self.healthy = True
        self.max_recoveries = 3
        self._recoveries = 0
        self._dead = False
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "prefill_s": 0.0, "decode_s": 0.0,
                      "speculative_tokens": 0, "speculative_kept": 0}
        self._calls = 0
        self.faults = dict(ecfg.faults)
        # "<call>:<kind>[@<tp rank>]": a fault restricted to one rank of a tensor-parallel group
        # (e.g. "0:k9-extra@0" desynchronises the group's K9 call counters)
        for item in filter(None, os.environ.get("ROUNDTABLE_ENGINE_FAULTS", "").split(",")):
            k, _, v = item.partition(":")
            v, _, only = v.strip().partition("@")
            if not only or int(only) == self.tp.rank:
                self.faults[int(k)] = v
        self.debug_checks = ecfg.debug_checks or os.environ.get("ROUNDTABLE_DEBUG_CHECKS") == "1"

    # ---- memory ----------------------------------------------------------------------------
    def _alloc_kv(self) -> PagedKVCache:
        m = self.model
        bs = self.ecfg.block_size
        per_block = PagedKVCache.bytes_per_block(self.cfg.n_layers, m.kv_heads_local, self.cfg.head_dim, bs,
                                                 torch.finfo(self.dtype).bits // 8)
        nb = self.ecfg.num_blocks
        if nb is None and self.ecfg.kv_budget_bytes is not None:
            nb = max(64, int(self.ecfg.kv_budget_bytes) // per_block)
        if nb is None:
            if self.on_gpu:
                free, _total = torch.cuda.mem_get_info(self.device)
                budget = int(free * self.ecfg.kv_cache_fraction) - (2 << 30)  # leave 2 GiB for activations
                nb = max(64, budget // per_block)
            else:
                nb = 256   # CPU plumbing runs: 8K resident tokens per engine
        if self.ecfg.max_kv_tokens:
            nb = min(nb, (self.ecfg.max_kv_tokens + bs - 1) // bs + self.ecfg.max_batch)
        if self.tp.size > 1:
            # every rank of a tensor-parallel knight must hold the SAME pool: the block allocator
            # then makes identical decisions on every rank, so a KVCacheOOM is raised on all of
            # them or none (a pool sized from one rank's free memory, e.g. a second rehearsal rank
            # on a shared GPU, could run out alone and skip collectives its peers enter)
            nb = self.tp.group_min(int(nb))
        kv = PagedKVCache(self.cfg.n_layers, m.kv_heads_local, self.cfg.head_dim, int(nb), bs,
                          self.device, self.dtype)
        kv.max_tokens = self.cfg.max_pos   # RoPE table / block-table width (_max_blocks)
        return kv

    def allocate_kv(self, budget_bytes: Optional[int] = None) -> None:
        """Deferred KV pool (``defer_kv``): sized by ``budget_bytes`` — EnginePool.finalize splits a
        GPU's free HBM between the engines placed on it once all their weights are resident."""
        if self._kv is None:
            if budget_bytes is not None:
                self.ecfg.kv_budget_bytes = int(budget_bytes)
            self._kv = self._alloc_kv()

    @property
    def kv(self) -> PagedKVCache:
        """The paged KV pool (allocated on first use when deferred)."""
        if self._kv is None:
            self.allocate_kv()
        return self._kv

    @property
    def kv_allocated(self) -> bool:
        return self._kv is not None

    def kv_bytes_per_token(self) -> int:
        return PagedKVCache.bytes_per_block(self.cfg.n_layers, self.model.kv_heads_local, self.cfg.head_dim, 1,
                                            torch.finfo(self.dtype).bits // 8)

    @property
    def kv_capacity_tokens(self) -> int:
        return self.kv.num_blocks * self.kv.block_size

    def max_source_chars(self) -> int:
        """Source budget in chars: positional limit minus response/overhead reserve (local-llm.ts:58-70)."""
        ctx = min(self.cfg.max_pos, self.kv_capacity_tokens)
        avail = max(ctx - 4096 - 3000, 2000)
        return int(avail * 4)

    # ---- tokenization ------------------------------------------------------------------------
    def _segment_ids(self, segs) -> List[Sequence[int]]:
        """Per-segment token ids: pinned ids as given (a list of ints is used without a copy),
        text through the tokenizer with a per-text cache."""
        fam = self.tokenizer.family
        res: List[Sequence[int]] = []
        for s in segs:
            if s.ids is not None and s.tokenizer == fam:
                res.append(s.ids if type(s.ids) is list else [int(i) for i in s.ids])
                continue
            key = (fam, s.text)
            ids = self._seg_cache.get(key)
            if ids is None:
                ids = self.tokenizer.encode(s.text)
                if len(self._seg_cache) > 4096:
                    self._seg_cache.clear()
                self._seg_cache[key] = ids
            res.append(ids)
        return res

    def encode_prompt(self, prompt: PromptLike) -> List[int]:
        return self._encode_segments(prompt, self._segment_ids(
            [Segment(prompt)] if isinstance(prompt, str) else prompt.segments))

    def _encode_segments(self, prompt: PromptLike, seg_ids: Sequence[Sequence[int]]) -> List[int]:
        out: List[int] = []
        for ids in seg_ids:
            out.extend(ids)
        pre, suf = self.tokenizer.chat_prefix, self.tokenizer.chat_suffix
        if (pre or suf) and not getattr(prompt, "templated", False):
            # constant wrap: the LCP reuse of the content is unaffected
            return list(pre) + out + list(suf)
        if not out:
            out = [self.tokenizer.bos_id]
        return out

    def encode_prompt_split(self, prompt: PromptLike) -> Tuple[List[int], int]:
        """Token ids plus the length of the prompt's shared part (``Prompt.shared_segments``
        leading segments, chat-template prefix included; 0 without a ``shared_key``)."""
        if isinstance(prompt, str):
            return self.encode_prompt(prompt), 0
        seg_ids = self._segment_ids(prompt.segments)
        ids = self._encode_segments(prompt, seg_ids)
        nseg = getattr(prompt, "shared_segments", 0) if getattr(prompt, "shared_key", None) else 0
        if nseg <= 0:
            return ids, 0
        n = sum(len(x) for x in seg_ids[:nseg])
        if n == 0 and seg_ids[:nseg]:      # an empty templated head encodes as [bos]
            n = 1
        pre = self.tokenizer.chat_prefix
        if pre and not getattr(prompt, "templated", False):
            n += len(pre)
        return ids, min(n, len(ids) - 1)

    # ---- prefix reuse ------------------------------------------------------------------------
    def sync_prefix(self, key: str, target: List[int]) -> Tuple[SeqState, int]:
        """Roll the resident sequence back to its LCP with ``target``; return (seq, reused tokens)."""
        s = self.kv.seq(key)
        n = lcp(s.tokens, target, len(target) - 1)   # always recompute >= 1 token (need its logits)
        self.kv.truncate(s, n)
        return s, n

    @staticmethod
    def shared_seq_key(key: str) -> str:
        return "@shared:" + key

    MAX_SHARED_SEQS = 64   # resident shared prefixes (tables, system prompts); LRU beyond

    def sync_shared(self, key: str, shared: List[int], protect=()) -> Tuple[SeqState, List[int]]:
        """Roll the table's shared sequence back to its LCP with ``shared``; return (seq, delta to
        prefill). The shared sequence is never decoded: it only holds the common KV blocks.
        Least-recently-used shared sequences beyond ``MAX_SHARED_SEQS`` are released (blocks a
        member still references stay alive through their refcount) — never one of ``protect``
        (the keys of the batch being set up, whose blocks its members have yet to attach)."""
        sk = self.shared_seq_key(key)
        lru = self.__dict__.setdefault("_shared_lru", {})
        lru.pop(sk, None)
        lru[sk] = None
        keep = {self.shared_seq_key(k) for k in protect} | {sk}
        while len(lru) > self.MAX_SHARED_SEQS:
            old = next((k for k in lru if k not in keep), None)
            if old is None:
                break
            del lru[old]
            self.kv.free_seq(old)
        s = self.kv.seq(sk)
        n = lcp(s.tokens, shared)
        spec = self.__dict__.setdefault("_spec_pred", {}).pop(sk, None)
        if spec is not None:   # how much of a speculative prefill the real prompt kept
            base, pred = spec
            self.stats["speculative_kept"] += max(0, min(n, len(pred)) - base)
        self.kv.truncate(s, n)
        return s, shared[n:]

    def attach_shared(self, s: SeqState, shared: SeqState, nblocks: int) -> int:
        """Make ``s`` start with the first ``nblocks`` FULL blocks of ``shared`` (refcounted, no
        copy): keep the leading blocks ``s`` already shares with it, drop the rest of ``s`` and
        reference the shared blocks beyond. Returns the shared token count. Writers copy-on-write
        a shared tail block, so a referenced block never changes under a reader."""
        bs = self.kv.block_size
        nblocks = min(nblocks, shared.length // bs)
        k = 0
        while k < min(len(s.blocks), nblocks) and s.blocks[k] == shared.blocks[k]:
            k += 1
        if k == nblocks and s.length >= nblocks * bs:
            # already holds every shared block (same ids = same K/V): keep the member's own tokens
            # past the shared region — sync_prefix rolls them back by LCP if they changed
            return nblocks * bs
        self.kv.truncate(s, min(s.length, k * bs))   # keeps <= k blocks, all shared ones
        for i in range(len(s.blocks), nblocks):
            self.kv.alloc.incref(shared.blocks[i])
            s.blocks.append(shared.blocks[i])
        s.tokens[:] = shared.tokens[:nblocks * bs]     # a referenced shared block is always full
        return nblocks * bs

    @torch.no_grad()
    def warm_shared(self, prompt: PromptLike) -> int:
        """Prefill the shared part of a PREDICTED next prompt into its table's shared sequence
        ahead of the turn (the C1 overlap, knights/distributed.py): the real turn's
        ``sync_shared`` keeps it by LCP, a wrong guess is rolled back the same way. KV only, no
        logits are used. Tensor-parallel engines never speculate (their ranks would have to
        agree on it). Returns the tokens prefilled."""
        key = getattr(prompt, "shared_key", None)
        if key is None or not self.healthy or self.tp.size > 1:
            return 0
        ids, n = self.encode_prompt_split(prompt)
        if n <= 0:
            return 0
        with self._on_stream():
            sq, delta = self.sync_shared(key, ids[:n])
            if not delta:
                return 0
            self._spec_pred[self.shared_seq_key(key)] = (n - len(delta), ids[:n])
            try:
                with trace.range(f"speculative shared prefill {len(delta)}"):
                    self.prefill_reserved([self.reserve(sq, delta)])
            except KVCacheOOM:
                self.kv.truncate(sq, len(ids[:n]) - len(delta))
                return 0
            except RuntimeError as e:
                # the reserved span's KV may be incomplete: drop the whole shared sequence (the
                # next turn prefills it again) and let run_turns' recovery probe the device
                sk = self.shared_seq_key(key)
                self.__dict__.get("_shared_lru", {}).pop(sk, None)
                self._spec_pred.pop(sk, None)
                self.kv.free_seq(sk)
                msg = str(e)
                if "HIP" in msg or "hip" in msg or "device" in msg:
                    self.healthy = False
                return 0
        self.stats["speculative_tokens"] += len(delta)
        self.stats["prefill_tokens"] += len(delta)
        return len(delta)

    def release(self, key: str) -> None:
        self.kv.free_seq(key)

    def fork(self, src: str, dst: str, copy: bool = False) -> None:
        self.kv.fork(src, dst, copy=copy)

    # ---- forward helpers -----------------------------------------------------------------------
    def _max_blocks(self) -> int:
        return (self.cfg.max_pos + self.kv.block_size - 1) // self.kv.block_size

    @torch.no_grad()
    def prefill(self, items: Sequence[Tuple[SeqState, List[int]]]) -> torch.Tensor:
        """Append ``ids`` to each sequence's KV (chunked, varlen-batched). Returns last-token logits [S, V]."""
        return self.prefill_reserved([self.reserve(s, ids) for s, ids in items])

    def reserve(self, s: SeqState, ids: Sequence[int]) -> Tuple[SeqState, int, List[int]]:
        """Append ``ids`` to ``s`` (tokens + KV blocks) ahead of their prefill: a shared
        prefix reserved this way can be attached to its members and prefilled in the SAME
        forward as their own deltas (items run in order; within a layer every K/V write
        precedes the attention that reads it)."""
        st = s.length
        ids = list(ids)
        self.kv.ensure_capacity(s, st + len(ids))
        s.tokens.extend(ids)
        return s, st, ids

    def prefill_reserved(self, items: Sequence[Tuple[SeqState, int, List[int]]]) -> torch.Tensor:
        """Compute the K/V of reserved spans (``reserve``) in order, chunked and varlen-batched;
        returns each span's last-token logits [S, V]."""
        dev = self.device
        pending = [(s, ids) for s, _, ids in items]
        base = [st for _, st, _ in items]
        last_logits: List[Optional[torch.Tensor]] = [None] * len(pending)
        offs = [0] * len(pending)
        budget = self.ecfg.prefill_chunk
        while True:
            batch = []
            used = 0
            for i, (s, ids) in enumerate(pending):
                rem = len(ids) - offs[i]
                if rem <= 0:
                    continue
                take = min(rem, max(1, budget - used))
                if used and used + take > budget:
                    break
                batch.append((i, take))
                used += take
                if used >= budget:
                    break
            if not batch:
                break
            seqs = []
            tok, pos, slots, cu, starts, last = [], [], [], [0], [], []
            for i, take in batch:
                s, ids = pending[i]
                st = base[i] + offs[i]
                chunk = ids[offs[i]:offs[i] + take]
                tok += chunk
                pos += list(range(st, st + take))
                slots += self.kv.slots(s, st, st + take)
                starts.append(st)
                cu.append(cu[-1] + take)
                last.append(cu[-1] - 1)
                offs[i] += take
                seqs.append(s)
            maxb = max(len(s.blocks) for s in seqs)
            bt = torch.zeros(len(seqs), maxb, dtype=torch.int32)
            for j, s in enumerate(seqs):
                bt[j, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
            cu_t = torch.tensor(cu, dtype=torch.int32)
            meta = AttnMeta(kind="prefill",
                            slot_mapping=torch.tensor(slots, dtype=torch.int64).to(dev, non_blocking=True),
                            block_tables=bt.to(dev, non_blocking=True),
                            cu_q=cu_t.to(dev, non_blocking=True),
                            start_pos=torch.tensor(starts, dtype=torch.int32).to(dev, non_blocking=True),
                            last_rows=torch.tensor(last, dtype=torch.int64).to(dev, non_blocking=True))
            if self.debug_checks:
                self.check_paging(bt, slots)
            if self.on_gpu:
                rows = ops.native().prefill_rows_per_tile(self.model.n_heads // self.model.n_kv_heads,
                                                          self.cfg.head_dim)
                meta.tile_map = ops.prefill_tile_map(cu_t, rows, torch.tensor(starts)).to(dev, non_blocking=True)
                # few tiles x KV heads (a tensor-parallel shard) leave most CUs idle: cut the long
                # tiles' key ranges into partials merged by a second launch (attention_prefill32.hip)
                G = self.model.n_heads // self.model.n_kv_heads
                if self.ecfg.prefill_key_split and ops.native().prefill_split_supported(G, self.cfg.head_dim):
                    plan = ops.prefill_split_plan(cu_t, rows, torch.tensor(starts), self.model.n_kv_heads)
                    if plan is not None:
                        meta.prefill_split = (plan[0].to(dev, non_blocking=True), plan[1].to(dev, non_blocking=True),
                                              plan[2])
            with trace.range("prefill"):
                logits = self.model.forward(torch.tensor(tok, dtype=torch.int64).to(dev, non_blocking=True),
                                            torch.tensor(pos, dtype=torch.int64).to(dev, non_blocking=True),
                                            self.kv, meta)
            for j, (i, take) in enumerate(batch):
                if offs[i] >= len(pending[i][1]):
                    last_logits[i] = logits[j]
        return torch.stack([l for l in last_logits])  # type: ignore[misc]

    # ---- the turn API ----------------------------------------------------------------------------
    @torch.no_grad()
    def run_turns(self, turns: Sequence[Turn]) -> List[TurnOutput]:
        """Run one turn for each entry (distinct seq_keys), batched; per-turn errors are returned."""
        if not turns:
            return []
        unhealthy = not self.healthy
        if self.tp.size > 1:
            # ranks of a TP knight decide together: one rank recovering into the prefill
            # collectives while another returns errors would hang the first
            unhealthy = self.tp.any_rank(unhealthy)
        if unhealthy and not self._recover():
            err = AdapterError("engine", "engine unhealthy after a previous device error", kind="device")
            return [TurnOutput("", [], {}, err) for _ in turns]
        call = self._calls
        self._calls += 1
        try:
            self._inject(call)
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    return self._run_turns(turns)
            return self._run_turns(turns)
        except KVCacheOOM as e:
            for t in turns:  # drop partial state; the knight re-prefills next time
                self.release(t.seq_key)
            return [TurnOutput("", [], {}, AdapterError("engine", f"out of memory: {e}", kind="oom")) for _ in turns]
        except EngineTimeout as e:
            return [TurnOutput("", [], {}, e) for _ in turns]
        except DeviceFlagError as e:
            # a bounded device-side wait expired: this turn's tokens are wrong. Fail the turn,
            # drop its KV (the knight re-prefills next turn) AND every shared-prefix sequence the
            # call prefilled — its all-reduces may have summed stale data, and sync_shared would
            # hand that KV to every member of the table by LCP. The engine itself stays usable:
            # an expiry the group agreed on (check_device_flags) may mean the ranks' K9 call
            # counters diverged, so the group re-agrees them before the next turn
            if getattr(e, "agreed", False):
                self._resync_k9()
            lru = self.__dict__.get("_shared_lru", {})
            for t in turns:
                self.release(t.seq_key)
                key = getattr(t.prompt, "shared_key", None)
                if key is not None:
                    sk = self.shared_seq_key(key)
                    lru.pop(sk, None)
                    self.kv.free_seq(sk)
            return [TurnOutput("", [], {}, AdapterError("engine", str(e), kind="device")) for _ in turns]
        except RuntimeError as e:
            msg = str(e)
            if "HIP" in msg or "hip" in msg or "CUDA" in msg or "device" in msg:
                self.healthy = False
                return [TurnOutput("", [], {}, AdapterError("engine", f"HIP error: {msg}", kind="device"))
                        for _ in turns]
            raise

    def _recover(self) -> bool:
        """Try to bring an unhealthy engine back: probe the device with a small
        kernel; if it answers, drop every resident sequence and captured graph (their state may
        be stale) and serve again — knights re-prefill from the transcript on their next turn.
        At most ``max_recoveries`` attempts per engine; a dead device stays unhealthy."""
        ok = not (self._recoveries >= self.max_recoveries or self._dead)
        if ok:
            self._recoveries += 1
            try:
                if self.on_gpu:
                    torch.cuda.synchronize(self.device)
                x = torch.ones(64, 64, device=self.device, dtype=torch.float32)
                ok = float((x @ x).sum().item()) == 64.0 ** 3
            except RuntimeError:
                ok = False
        if self.tp.size > 1:
            ok = not self.tp.any_rank(not ok)   # the whole group recovers, or none of it
        if not ok:
            self.healthy = False
            return False
        for key in list(self.kv.seqs):
            self.kv.free_seq(key)
        self.graphs.clear()
        # the failed work may have left the ranks' K9 call counters apart (calls one rank issued
        # alone): the recovered group starts from one agreed epoch
        self._resync_k9()
        self.healthy = True
        return True

    def _inject(self, call: int) -> None:
        f = self.faults.get(call)
        if f is None:
            return
        if f == "oom":
            raise KVCacheOOM(f"injected KV-cache exhaustion at call {call}")
        if f == "timeout":
            raise EngineTimeout("engine", f"injected timeout at call {call}")
        if f == "device":
            raise RuntimeError(f"HIP error: injected device fault at call {call}")
        if f == "device-dead":      # a fault the recovery probe cannot clear
            self._dead = True
            raise RuntimeError(f"HIP error: injected unrecoverable device fault at call {call}")
        if f == "flag":             # a bounded device-side wait expired (K9 / persistent kernel)
            raise DeviceFlagError("engine", f"injected poll expiry at call {call}", kind="device")
        if f == "k9-extra":         # one K9 call on THIS rank alone: the group's call counters diverge
            os_ = self.tp.oneshot
            if os_ is not None:
                with self._on_stream():   # in order with the turn's own calls (one call at a time per comm)
                    os_(torch.zeros(os_.world * 64, dtype=torch.bfloat16, device=self.device))
            return
        raise AdapterError("engine", f"injected failure at call {call}", kind="unknown")

    def check_paging(self, block_tables: torch.Tensor, slots: Sequence[int]) -> None:
        """Debug-mode bounds asserts on the paging metadata a kernel is about to dereference."""
        nb = self.kv.num_blocks
        bt = block_tables.cpu()
        if bt.numel() and (int(bt.min()) < 0 or int(bt.max()) >= nb):
            raise AssertionError(f"block table entry outside [0, {nb}): {int(bt.min())}..{int(bt.max())}")
        lim = nb * self.kv.block_size
        bad = [x for x in slots if x < 0 or x >= lim]
        if bad:
            raise AssertionError(f"slot mapping outside [0, {lim}): {bad[:4]}")

    def _run_turns(self, turns: Sequence[Turn]) -> List[TurnOutput]:
        # members of one shared-prefix group must be adjacent in the decode batch
        order = group_order([getattr(t.prompt, "shared_key", None) for t in turns])
        if order == list(range(len(turns))):
            return self._run_turns_ordered(turns)
        outs = self._run_turns_ordered([turns[i] for i in order])
        res: List[Optional[TurnOutput]] = [None] * len(turns)
        for j, i in enumerate(order):
            res[i] = outs[j]
        return res  # type: ignore[return-value]

    def _sync_groups(self, turns: Sequence[Turn], enc: Sequence[Tuple[List[int], int]]):
        """Reserve every shared-prefix group's new common tokens ONCE in the group's shared
        sequence and attach its full blocks to each member (``prompt_layout: shared``); the
        caller prefills the reserved spans first in the members' forward.
        Returns (per-turn group key or None, {key: shared seq}, {key: shared prefill tokens},
        reserved shared spans)."""
        keys = [getattr(t.prompt, "shared_key", None) if n > 0 else None for t, (_, n) in zip(turns, enc)]
        shared: Dict[str, SeqState] = {}
        pre: Dict[str, int] = {}
        items = []
        batch_keys = [k for k in dict.fromkeys(keys) if k is not None]
        for key in batch_keys:
            members = [i for i, k in enumerate(keys) if k == key]
            common = enc[members[0]][0][:enc[members[0]][1]]
            for i in members[1:]:
                common = common[:lcp(common, enc[i][0], enc[i][1])]
            sq, delta = self.sync_shared(key, common, protect=batch_keys)
            shared[key] = sq
            pre[key] = len(delta)
            if delta:
                items.append(self.reserve(sq, delta))   # KV only; never sampled
        bs = self.kv.block_size
        for t, key in zip(turns, keys):
            if key is not None:
                sq = shared[key]
                self.attach_shared(self.kv.seq(t.seq_key), sq, sq.length // bs)
        return keys, shared, pre, items

    def _prefill_turns(self, shared_items, seqs: Sequence[SeqState], deltas: Sequence[List[int]]) -> torch.Tensor:
        """One prefill over the reserved shared spans, then every turn's own delta; returns the
        turns' last-token logits."""
        logits = self.prefill_reserved(list(shared_items) + [self.reserve(s, d) for s, d in zip(seqs, deltas)])
        return logits[len(shared_items):]

    def _run_turns_ordered(self, turns: Sequence[Turn]) -> List[TurnOutput]:
        t_start = time.perf_counter()
        enc = [self.encode_prompt_split(t.prompt) for t in turns]
        targets = [ids for ids, _ in enc]
        self._sync()
        t0 = time.perf_counter()
        keys, shared, shared_pre, shared_items = self._sync_groups(turns, enc)
        seqs, reused = [], []
        for t, ids in zip(turns, targets):
            s, n = self.sync_prefix(t.seq_key, ids)
            seqs.append(s)
            reused.append(n)
        deltas = [ids[n:] for ids, n in zip(targets, reused)]
        logits = self._prefill_turns(shared_items, seqs, deltas)
        first = self._sample_host(logits, seqs, turns)
        # blocks every member of a group still shares (a member rolled back into the shared
        # region has copied-on-write its tail): the grouped decode reads those once per group
        sh_blocks: Dict[str, int] = {}
        for s, key in zip(seqs, keys):
            if key is not None:
                sh_blocks[key] = min(sh_blocks.get(key, 1 << 30), common_blocks(s, shared[key]))
        groups = ([k if k is not None and sh_blocks[k] > 0 else None for k in keys],
                  [sh_blocks.get(k, 0) if k is not None else 0 for k in keys])
        self._sync()
        t1 = time.perf_counter()
        gen, decode_steps = self.decode(seqs, turns, first, deadline=t_start + min(t.timeout_s for t in turns),
                                        groups=groups if any(g is not None for g in groups[0]) else None)
        forced = self._force_tails(seqs, turns, gen)
        self._sync()
        t2 = time.perf_counter()
        self.check_device_flags()
        outs = []
        seen = set()
        dev_gen = getattr(self, "_dev_gen", None) or [None] * len(turns)
        for t, s, g, n, d, key, nf, dg in zip(turns, seqs, gen, reused, deltas, keys, forced, dev_gen):
            text = self.tokenizer.decode(g)
            spre = 0
            if key is not None and key not in seen:     # the group's shared prefill, counted once
                seen.add(key)
                spre = shared_pre[key]
            outs.append(TurnOutput(text, g, {
                "prompt_tokens": len(d) + n, "prefill_tokens": len(d) + spre, "reused_tokens": n,
                "shared_tokens": sh_blocks.get(key, 0) * self.kv.block_size if key is not None else 0,
                "decode_tokens": len(g) - nf, "forced_tokens": nf, "prefill_ms": (t1 - t0) * 1e3,
                "decode_ms": (t2 - t1) * 1e3, "decode_tok_s": (len(g) - nf) / max(t2 - t1, 1e-9), "batch": len(turns),
                "resident_tokens": s.length, "turn_ms": (t2 - t_start) * 1e3, "tp": self.tp.size},
                dev_ids=dg if nf == 0 else None))   # forced tails exist only on the host
        self.stats["prefill_tokens"] += sum(len(d) for d in deltas) + sum(shared_pre.values())
        self.stats["decode_tokens"] += sum(len(g) for g in gen) - sum(forced)
        self.stats["prefill_s"] += t1 - t0
        self.stats["decode_s"] += t2 - t1
        return outs

    def _force_tails(self, seqs: Sequence[SeqState], turns: Sequence[Turn], gen: List[List[int]]) -> List[int]:
        """Teacher-force ``params.forced_tail`` after each turn's sampled tokens (scripted
        consensus): prefill it like generated text, so the resident KV covers the whole reply
        except its last token, as after a normal decode."""
        items, counts = [], []
        for s, t, g in zip(seqs, turns, gen):
            if not t.params.forced_tail:
                counts.append(0)
                continue
            tail = self.tokenizer.encode(t.params.forced_tail)
            feed = ([g[-1]] if g else []) + tail[:-1]
            g.extend(tail)
            counts.append(len(tail))
            if feed:
                items.append((s, feed))
        if items:
            with trace.range("forced tail"):
                self.prefill(items)
        return counts

    def _sync(self):
        if self.on_gpu:
            # this engine's stream only: another engine on the same GPU keeps running
            (self.stream or torch.cuda.current_stream(self.device)).synchronize()

    def device_flag_errors(self) -> List[str]:
        """Read (and clear) the poll-expiry flag of the bounded device-side wait of the K9 one-shot
        all-reduce (a peer's flag). A set flag means the kernel proceeded on stale data, so the
        turn's output is wrong."""
        msgs: List[str] = []
        if not self.on_gpu:
            return msgs
        os_ = self.tp.oneshot
        if os_ is not None and os_.error() > 0:
            os_.clear_error()
            msgs.append("K9 one-shot all-reduce: a peer's flag never arrived (poll expired)")
        return msgs

    def check_device_flags(self) -> None:
        msgs = self.device_flag_errors()
        if self.tp.any_rank(bool(msgs)):     # every rank of a TP knight fails the turn together
            err = DeviceFlagError("engine", "; ".join(msgs) or "a peer rank's device wait expired",
                                  kind="device")
            err.agreed = True
            raise err

    def _resync_k9(self) -> None:
        """Collective over the TP group (every rank calls it at the same point): re-agree the K9
        call counter (:meth:`OneShotAllReduce.resync`). If any rank cannot, the group drops K9
        together — RCCL / host collectives from then on, and (a gloo rehearsal group, whose
        captured step needs K9) eager decode; captured graphs referencing the comm are dropped."""
        os_ = self.tp.oneshot
        if self.tp.size == 1 or os_ is None or not self.on_gpu:
            return
        self.stats["k9_resyncs"] = self.stats.get("k9_resyncs", 0) + 1
        if os_.resync():
            return
        import warnings
        warnings.warn("K9 one-shot comm could not be re-armed on every rank: the group falls back to "
                      "process-group collectives")
        os_.close()
        self.tp.oneshot = None
        self.graphs.clear()
        if self.tp.backend() != "nccl":
            self.ecfg.use_graphs = False

    # ---- continuous batching (serve.py): admit / step in chunks / retire ----------------------------
    def _on_stream(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    @torch.no_grad()
    def start_turns(self, turns: Sequence[Turn]) -> List[Tuple[SeqState, int, Dict[str, float]]]:
        with self._on_stream():
            return self._start_turns(turns)

    def _start_turns(self, turns: Sequence[Turn]) -> List[Tuple[SeqState, int, Dict[str, float]]]:
        """Prefill ``turns`` (LCP reuse, delta only) and sample each first token, WITHOUT decoding:
        returns (sequence, first token, metrics). The first token's K/V is not in the cache yet —
        it is the input of the next :meth:`continue_decode`."""
        enc = [self.encode_prompt_split(t.prompt) for t in turns]
        targets = [ids for ids, _ in enc]
        t0 = time.perf_counter()
        keys, _shared, shared_pre, shared_items = self._sync_groups(turns, enc)   # shared prefixes
        seqs, reused = [], []
        for t, ids in zip(turns, targets):
            sq, n = self.sync_prefix(t.seq_key, ids)
            seqs.append(sq)
            reused.append(n)
        deltas = [ids[n:] for ids, n in zip(targets, reused)]
        logits = self._prefill_turns(shared_items, seqs, deltas)
        first = self._sample_host(logits, seqs, turns).tolist()
        ms = (time.perf_counter() - t0) * 1e3
        self.stats["prefill_tokens"] += sum(len(d) for d in deltas) + sum(shared_pre.values())
        self.stats["prefill_s"] += ms / 1e3
        return [(sq, int(f), {"prompt_tokens": len(d) + n, "prefill_tokens": len(d), "reused_tokens": n,
                              "prefill_ms": ms}) for sq, f, d, n in zip(seqs, first, deltas, reused)]

    def decode_groups_for(self, seqs: Sequence[SeqState], turns: Sequence[Turn]):
        """(labels, shared blocks) of a decode batch from its turns' ``shared_key``s, or None:
        sequences still holding their group's shared blocks decode them once per group."""
        labels, blocks = [], []
        for sq, t in zip(seqs, turns):
            key = getattr(t.prompt, "shared_key", None)
            sh = self.kv.seqs.get(self.shared_seq_key(key)) if key else None
            nb = common_blocks(sq, sh) if sh is not None else 0
            labels.append(key if nb > 0 else None)
            blocks.append(nb)
        for key in set(l for l in labels if l is not None):   # a group shares its members' minimum
            m = min(b for l, b in zip(labels, blocks) if l == key)
            blocks = [m if l == key else b for l, b in zip(labels, blocks)]
        if not any(l is not None for l in labels):
            return None
        return labels, blocks

    @torch.no_grad()
    def continue_decode(self, seqs: Sequence[SeqState], turns: Sequence[Turn], last: Sequence[int],
                        steps: int) -> List[List[int]]:
        with self._on_stream():
            return self._continue_decode(seqs, turns, last, steps)

    def _continue_decode(self, seqs: Sequence[SeqState], turns: Sequence[Turn], last: Sequence[int],
                         steps: int) -> List[List[int]]:
        """Decode ``steps`` new tokens for every sequence of a (possibly changing) batch, given each
        sequence's last sampled token (not yet in the KV cache). Afterwards the cache holds every
        token except the newest one, so calls chain chunk by chunk while sequences join and leave."""
        if not seqs:
            return []
        order = group_order([getattr(t.prompt, "shared_key", None) for t in turns])
        if order != list(range(len(seqs))):     # group members adjacent in the batch
            outs = self._continue_decode([seqs[i] for i in order], [turns[i] for i in order],
                                         [last[i] for i in order], steps)
            res: List[List[int]] = [[] for _ in seqs]
            for j, i in enumerate(order):
                res[i] = outs[j]
            return res
        groups = self.decode_groups_for(seqs, turns)
        first = torch.tensor(list(last), dtype=torch.int64, device=self.device)
        for sq in seqs:
            self.kv.ensure_capacity(sq, sq.length + steps + 1)
        chunk = [Turn(t.seq_key, t.prompt, SamplingParams(**{**t.params.__dict__, "max_new_tokens": steps + 1,
                                                              "ignore_eos": True, "stop_on_consensus": False}),
                      t.timeout_s) for t in turns]
        eos = self.tokenizer.stop_ids
        t0 = time.perf_counter()
        runner = self._agreed_graph(len(seqs), max(sq.length for sq in seqs) + steps + 1, groups is not None,
                                    self.dist_greedy(chunk))
        with trace.range(f"decode chunk B={len(seqs)} steps={steps}"):
            if runner is not None:
                toks = runner.run(self, seqs, chunk, first, steps + 1, time.perf_counter() + 1e9, eos, groups)
            else:
                toks = self._decode_eager(seqs, chunk, first, steps + 1, time.perf_counter() + 1e9, eos, groups)
        out = []
        for sq, tk, f in zip(seqs, toks, last):
            new = list(tk[1:steps + 1])
            sq.tokens.extend([int(f)] + new[:-1])     # K/V now covers the old last token + all but the newest
            out.append(new)
        self.stats["decode_tokens"] += sum(len(n) for n in out)
        self.stats["decode_s"] += time.perf_counter() - t0
        return out

    def _sample_host(self, logits: torch.Tensor, seqs: Sequence[SeqState], turns: Sequence[Turn]) -> torch.Tensor:
        B = logits.shape[0]
        dev = logits.device
        temp = torch.tensor([t.params.temperature for t in turns], dtype=torch.float32, device=dev)
        top_p = torch.tensor([t.params.top_p for t in turns], dtype=torch.float32, device=dev)
        top_k = torch.tensor([t.params.top_k for t in turns], dtype=torch.int32, device=dev)
        seeds = torch.tensor([t.params.seq_seed(t.seq_key) for t in turns], dtype=torch.int64, device=dev)
        offs = torch.tensor([s.length for s in seqs], dtype=torch.int64, device=dev)
        return ops.sample(logits.contiguous(), temp, top_p, top_k, seeds, offs)

    # ---- decode -------------------------------------------------------------------------------------
    def decode(self, seqs: Sequence[SeqState], turns: Sequence[Turn], first: torch.Tensor,
               deadline: float, groups=None) -> Tuple[List[List[int]], int]:
        """``groups``: optional (per-sequence group key or None, per-sequence shared block count)
        — consecutive sequences of one key decode their shared KV blocks once (grouped K3)."""
        B = len(seqs)
        max_new = [max(1, t.params.max_new_tokens) for t in turns]
        steps = max(max_new)
        # every sequence: the first sampled token is "generated", then steps-1 decode forwards
        for s, n in zip(seqs, max_new):
            self.kv.ensure_capacity(s, s.length + steps)
        eos = self.tokenizer.stop_ids
        runner = self._agreed_graph(B, max(s.length for s in seqs) + steps, groups is not None, self.dist_greedy(turns))
        with trace.range(f"decode B={B} steps={steps}"):
            if runner is not None:
                toks = runner.run(self, seqs, turns, first, steps, deadline, eos, groups)
                dev_toks = runner.last_dev
            else:
                toks = self._decode_eager(seqs, turns, first, steps, deadline, eos, groups)
                dev_toks = None
        gen: List[List[int]] = []
        self._dev_gen: List[Optional[torch.Tensor]] = []
        for b, (s, t) in enumerate(zip(seqs, turns)):
            g = toks[b][:max_new[b]]
            if not t.params.ignore_eos:
                g = cut_at_stop(g, eos)
            if t.params.stop_on_consensus:
                g = _cut_at_consensus(self.tokenizer, g)
            gen.append(g)
            # the kept ids are a prefix of the sampled ones: their device copy is a slice
            self._dev_gen.append(dev_toks[b, :len(g)] if dev_toks is not None and len(g) <= dev_toks.shape[1]
                                 else torch.tensor(g, dtype=torch.int64).to(self.device, non_blocking=True))
            # resident KV = prompt + the tokens actually kept (the last one's K/V is not computed yet)
            # resident = prompt + kept tokens except the last (its K/V was never computed)
            s.tokens.extend(g)
            self.kv.truncate(s, s.length - 1 if g else s.length)
        if self.on_gpu:
            # the device ids are produced on this engine's stream; consumers on other streams (the
            # C1 exchange) wait on this event before reading them (parallel/exchange.py)
            ev = torch.cuda.Event()
            ev.record(self.stream or torch.cuda.current_stream(self.device))
            for d in self._dev_gen:
                d.ready_event = ev
        return gen, steps

    def group_table(self, groups, B: int) -> Optional[torch.Tensor]:
        """Host ``[B, 3]`` int32 group table for the grouped decode kernel (rows past the real
        sequences run alone), or None without groups."""
        if groups is None:
            return None
        labels, shb = list(groups[0]), list(groups[1])
        labels += [None] * (B - len(labels))
        shb += [0] * (B - len(shb))
        t, _ = ops.decode_groups(labels, shb, self.model.n_heads // self.model.n_kv_heads)
        return t

    def _decode_eager(self, seqs, turns, first, steps, deadline, eos, groups=None) -> List[List[int]]:
        dev = self.device
        B = len(seqs)
        cur = first.clone()
        out: List[List[int]] = [[int(x)] for x in cur.tolist()]
        lens = [s.length for s in seqs]
        temp = torch.tensor([t.params.temperature for t in turns], dtype=torch.float32, device=dev)
        top_p = torch.tensor([t.params.top_p for t in turns], dtype=torch.float32, device=dev)
        top_k = torch.tensor([t.params.top_k for t in turns], dtype=torch.int32, device=dev)
        seeds = torch.tensor([t.params.seq_seed(t.seq_key) for t in turns], dtype=torch.int64, device=dev)
        done = [False] * B
        bt = torch.zeros(B, max(len(s.blocks) for s in seqs), dtype=torch.int32)
        for j, s in enumerate(seqs):
            bt[j, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
        bt = bt.to(dev)
        bucket = next((b for b in BATCH_BUCKETS if b >= B), B)
        splits = ops.decode_splits(bucket, self.model.n_kv_heads, grouped=groups is not None) if self.on_gpu else 1
        G = self.model.n_heads // self.model.n_kv_heads
        ws = ops.DecodeWorkspace(B, self.model.n_heads, self.cfg.head_dim, splits, dev,
                                 max_group=ops.MAX_GROUP_COLS // G if groups is not None else 1) if self.on_gpu else None
        gt = self.group_table(groups, B)
        gt = gt.to(dev) if gt is not None and self.on_gpu else None
        dist_greedy = self.dist_greedy(turns)
        for step in range(1, steps):
            pos = list(lens)
            slots = [s.blocks[p // self.kv.block_size] * self.kv.block_size + p % self.kv.block_size
                     for s, p in zip(seqs, pos)]
            meta = AttnMeta(kind="decode", slot_mapping=torch.tensor(slots, dtype=torch.int64, device=dev),
                            block_tables=bt, ctx_lens=torch.tensor([p + 1 for p in pos], dtype=torch.int32, device=dev),
                            num_splits=splits, workspace=ws, groups=gt, local_logits=dist_greedy)
            logits = self.model.forward(cur.to(dev), torch.tensor(pos, dtype=torch.int64, device=dev), self.kv, meta)
            offs = torch.tensor([p + 1 for p in pos], dtype=torch.int64, device=dev)
            if dist_greedy:
                cur = self.tp.greedy_gather(logits, self.cfg.vocab)
            else:
                cur = ops.sample(logits.contiguous(), temp, top_p, top_k, seeds, offs)
            for b, x in enumerate(cur.tolist()):
                out[b].append(int(x))
            lens = [l + 1 for l in lens]
            if step % self.ecfg.sync_every == 0:
                if self.past_deadline(deadline, step // self.ecfg.sync_every):
                    self._unwind(seqs)
                    raise EngineTimeout("engine", "turn exceeded timeout_per_turn_seconds")
                done = [d or _finished(o, t.params, eos, self.tokenizer) for d, o, t in zip(done, out, turns)]
                if all(done):
                    break
        return out

    DEADLINE_AGREE_EVERY = 8   # tensor-parallel groups agree on the turn deadline every 8th check

    def past_deadline(self, deadline: float, check: int) -> bool:
        """The decode loop's wall-clock check (every chunk). A tensor-parallel group must stop at
        the SAME step on every rank — one rank leaving the loop alone would leave its peers'
        remaining K9 calls unanswered — so its ranks decide together, every
        ``DEADLINE_AGREE_EVERY``-th check (one small collective per ~256 steps; the turn may
        overrun its limit by that many steps)."""
        if self.tp.size == 1:
            return time.perf_counter() > deadline
        if check % self.DEADLINE_AGREE_EVERY:
            return False
        return self.tp.any_rank(time.perf_counter() > deadline)

    def _unwind(self, seqs):
        # the knights' tokens were not extended; drop the blocks pre-allocated for generation
        for s in seqs:
            self.kv.truncate(s, s.length)

    def dist_greedy(self, turns: Sequence[Turn]) -> bool:
        """TP knight decoding greedily: C3 moves (value, id) per rank instead of the logits —
        except in a captured step over a gloo group, where that host-staged gather cannot run:
        there the logits go through K9's one-shot gather and the sampler takes the argmax."""
        if self.tp.size == 1 or not all(t.params.temperature <= 0 for t in turns):
            return False
        return not (self.on_gpu and self.ecfg.use_graphs and self.tp.backend() != "nccl")

    def k9_only_step(self) -> bool:
        """Every collective of a decode step runs as a device-side K9 kernel: the all-reduces
        (K9 / fused EPI_AR) and the vocab gather (one-shot gather)."""
        os_ = self.tp.oneshot
        return os_ is not None and bool(getattr(os_, "gather_ok", False))

    def _agreed_graph(self, B: int, max_ctx: int, grouped: bool, dist_greedy: bool):
        """The captured decode step, or None (eager). A capture that fails on ANY rank of a
        tensor-parallel group sends EVERY rank to eager decode: a rank replaying a graph whose K9
        calls no peer issues would wait out each poll bound. The group agrees twice, only when the
        graph is not cached (cache keys are the same on every rank, so all ranks miss together and
        a cached replay costs no host round trip): after the graph's buffers are allocated (where
        an out-of-memory rank fails, before any K9 call) and after the capture itself, whose eager
        warm-up runs issue K9 calls — a rank failing in there leaves the counters apart, so the
        fallback re-agrees them (:meth:`_resync_k9`)."""
        if not (self.on_gpu and self.ecfg.use_graphs):
            return None
        key = self._graph_key(B, grouped, dist_greedy)
        g = self.graphs.get(key)
        if g is not None:
            return g
        from .graphs import DecodeGraph
        g, err = None, None
        try:
            with failsafe.stage("capture"):
                g = DecodeGraph(self, key[0], key[1], grouped=grouped, dist_greedy=dist_greedy, capture=False)
        except RuntimeError as e:   # out of memory for the graph's static buffers
            err = e
        failed = self.tp.any_rank(err is not None) if self.tp.size > 1 else err is not None
        calls_issued = False
        if not failed:
            try:
                with failsafe.stage("capture"):
                    calls_issued = True
                    g.capture()
            except RuntimeError as e:   # e.g. a collective that refuses stream capture
                err = e
            failed = self.tp.any_rank(err is not None) if self.tp.size > 1 else err is not None
        if failed:
            if self.tp.size == 1:
                raise err
            import warnings
            warnings.warn(f"hipGraph capture failed on a rank of the tp={self.tp.size} group "
                          f"({err if err is not None else 'peer rank'}); every rank decodes eagerly")
            self.ecfg.use_graphs = False
            self.graphs.clear()
            self.stats["capture_fallbacks"] = self.stats.get("capture_fallbacks", 0) + 1
            if calls_issued:
                self._resync_k9()
            return None
        self.graphs[key] = g
        return g

    def _graph_key(self, B: int, grouped: bool, dist_greedy: bool) -> Tuple[int, int, bool, bool]:
        bucket = next((b for b in BATCH_BUCKETS if b >= B), B)
        return (bucket, ops.decode_splits(bucket, self.model.n_kv_heads, grouped=grouped), grouped, dist_greedy)

    def _graph_for(self, B: int, max_ctx: int, grouped: bool = False, dist_greedy: bool = False) -> "DecodeGraph":
        from .graphs import DecodeGraph
        key = self._graph_key(B, grouped, dist_greedy)
        g = self.graphs.get(key)
        if g is None:
            g = DecodeGraph(self, key[0], key[1], grouped=grouped, dist_greedy=dist_greedy)
            self.graphs[key] = g
        return g


def lcp(a: Sequence[int], b: Sequence[int], lim: Optional[int] = None) -> int:
    """Length of the common prefix of ``a`` and ``b`` (at most ``lim``). Compares 4K-token
    slices in C first (a 40K-token transcript: ~0.2 ms instead of ~8 ms element by element)."""
    lim = min(len(a), len(b)) if lim is None else min(lim, len(a), len(b))
    lo = 0
    while lo < lim:
        hi = min(lim, lo + 4096)
        if a[lo:hi] != b[lo:hi]:        # (also for equal values in different sequence types)
            while lo < hi and a[lo] == b[lo]:
                lo += 1
            if lo < hi:
                return lo
        lo = hi
    return lim


def common_blocks(s: SeqState, shared: SeqState) -> int:
    """Leading blocks ``s`` references from ``shared`` (same ids, hence same K/V)."""
    k, lim = 0, min(len(s.blocks), len(shared.blocks))
    while k < lim and s.blocks[k] == shared.blocks[k]:
        k += 1
    return k


def group_order(keys: Sequence[Optional[str]]) -> List[int]:
    """Stable permutation putting turns with the same shared-prefix key next to each other
    (first appearance order); key-less turns keep their relative place."""
    first: Dict[object, int] = {}
    for i, k in enumerate(keys):
        first.setdefault(k if k is not None else ("__alone", i), i)
    return sorted(range(len(keys)), key=lambda i: (first[keys[i] if keys[i] is not None else ("__alone", i)], i))


def cut_at_stop(ids: List[int], stops: frozenset) -> List[int]:
    """Keep ``ids`` up to and including the first end-of-turn id (``tokenizer.stop_ids``)."""
    for j, i in enumerate(ids):
        if i in stops:
            return ids[:j + 1]
    return ids


def _finished(out: List[int], params: SamplingParams, eos: frozenset, tok: EngineTokenizer) -> bool:
    """``eos``: the tokenizer's stop-id set."""
    if len(out) >= params.max_new_tokens:
        return True
    if not params.ignore_eos and not eos.isdisjoint(out):
        return True
    if params.stop_on_consensus and len(out) > 8:
        return _consensus_closed(tok, out)
    return False


def _consensus_closed(tok: EngineTokenizer, ids: List[int]) -> bool:
    text = tok.decode(ids)
    return "consensus_score" in text and parse_consensus(text, "", 0) is not None


def _cut_at_consensus(tok: EngineTokenizer, ids: List[int]) -> List[int]:
    """Truncate right after the first complete consensus block (decode may overshoot by < sync_every)."""
    text = tok.decode(ids)
    if "consensus_score" not in text or parse_consensus(text, "", 0) is None:
        return ids
    lo, hi = 1, len(ids)
    while lo < hi:  # smallest prefix that still parses
        mid = (lo + hi) // 2
        if parse_consensus(tok.decode(ids[:mid]), "", 0) is not None:
            hi = mid
        else:
            lo = mid + 1
    return ids[:lo]
