"""hipGraph-captured decode step (one replay = one token for every knight in the batch).

The captured region is the whole step: embedding, all layers (K1/K2/K3/K5 + GEMMs
+ TP all-reduces), lm_head, K6 sampling, then device-side bookkeeping so the next
replay needs no host input: the sampled ids become the next inputs, positions /
context lengths / the step counter advance, and the next slot mapping, sampler
offsets and embedding rows are derived from the (pre-allocated) block tables in the
same launch (fused path: csrc/decode_step.hip decode_advance with prep operands; the
turn's first step is prepped once, eagerly, before the first replay). Static buffers
are refreshed once per turn.

Graphs are cached per (batch bucket, split-KV count); padded batch rows decode a
dummy sequence living in a reserved scratch block and are discarded.
"""
from __future__ import annotations

import contextlib
import gc
import threading
import time
from typing import List, Sequence

import torch

from .. import ops
from ..errors import EngineTimeout
from ..models.llama import AttnMeta

MAX_STEPS = 8192

_gc_lock = threading.Lock()
_gc_depth = 0
_gc_was_enabled = False


@contextlib.contextmanager
def no_gc_during_capture():
    """Python's cyclic collector off while any thread captures a graph: the first capture to
    enter collects and disables it, the last one to leave restores the state found on entry."""
    global _gc_depth, _gc_was_enabled
    with _gc_lock:
        if _gc_depth == 0:
            gc.collect()
            _gc_was_enabled = gc.isenabled()
            gc.disable()
        _gc_depth += 1
    try:
        yield
    finally:
        with _gc_lock:
            _gc_depth -= 1
            if _gc_depth == 0 and _gc_was_enabled:
                gc.enable()


class DecodeGraph:
    def __init__(self, engine, bucket: int, splits: int, grouped: bool = False, dist_greedy: bool = False,
                 capture: bool = True):
        self.engine = engine
        self.B = bucket
        self.splits = splits
        self.dist_greedy = dist_greedy   # TP greedy: C3 all-gathers (value, id) per rank, not logits
        dev = engine.device
        kv = engine.kv
        self.bs = kv.block_size
        self.maxb = engine._max_blocks()
        if not hasattr(engine, "_scratch_block"):
            engine._scratch_block = kv.alloc.alloc()
        self.scratch = engine._scratch_block
        B = bucket
        self.input_ids = torch.zeros(B, dtype=torch.int64, device=dev)
        self.positions = torch.zeros(B, dtype=torch.int64, device=dev)
        self.ctx_lens = torch.ones(B, dtype=torch.int32, device=dev)
        self.block_tables = torch.full((B, self.maxb), self.scratch, dtype=torch.int32, device=dev)
        self.temp = torch.zeros(B, dtype=torch.float32, device=dev)
        self.top_p = torch.ones(B, dtype=torch.float32, device=dev)
        self.top_k = torch.zeros(B, dtype=torch.int32, device=dev)
        self.seeds = torch.zeros(B, dtype=torch.int64, device=dev)
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.out = torch.zeros(MAX_STEPS, B, dtype=torch.int64, device=dev)
        self.slots = torch.zeros(B, dtype=torch.int64, device=dev)
        self.offsets = torch.zeros(B, dtype=torch.int64, device=dev)
        self.hidden = torch.zeros(B, engine.model.cfg.hidden, dtype=engine.model.dtype, device=dev)
        G = engine.model.n_heads // engine.model.n_kv_heads
        self.ws = ops.DecodeWorkspace(B, engine.model.n_heads, engine.cfg.head_dim, max(1, splits), dev,
                                      max_group=ops.MAX_GROUP_COLS // G if grouped else 1)
        # shared-prefix group table (grouped K3); rows default to "alone"
        self.groups = None
        if grouped:
            self.groups = torch.zeros(B, 3, dtype=torch.int32, device=dev)
            self._reset_groups()
        self.guard_err = torch.zeros(1, dtype=torch.int32, device=dev)   # debug paging guard (captured)
        self.nxt = torch.zeros(B, dtype=torch.int64, device=dev)
        self.sample_ws = ops.sample_workspace(B, dev)      # self-re-arming K6 tickets
        self.graph = None
        self._host_out: List[torch.Tensor] = []
        if capture:     # (Engine._agreed_graph agrees on the buffers first, then captures)
            self._capture()

    def capture(self) -> None:
        self._capture()

    def _fused(self) -> bool:
        m = self.engine.model
        return getattr(m, "accepts_hidden", False) and m.fused_decode_ok(self.input_ids)

    def _prep(self):
        """Eager prologue of a turn's first step: K/V slots, sampler offsets, embedding rows.
        Later steps get theirs from the previous step's decode_advance."""
        if self._fused():
            ops.decode_prep(self.slots, self.offsets, self.hidden, self.input_ids, self.positions,
                            self.block_tables, self.engine.model.w["embed"], self.bs)

    def _body(self):
        e = self.engine
        fused = self._fused()
        if fused:
            slots, offsets, hidden = self.slots, self.offsets, self.hidden
        else:
            bs = self.bs
            blk = self.block_tables.gather(1, (self.positions // bs).unsqueeze(1)).squeeze(1).long()
            slots = blk * bs + self.positions % bs
            offsets, hidden = self.positions + 1, None
        if e.debug_checks:   # device-side bounds asserts on what this step's kernels dereference
            ops.paging_guard(self.block_tables, self.ctx_lens, self.positions, slots, self.guard_err,
                             e.kv.num_blocks, self.bs)
        meta = AttnMeta(kind="decode", slot_mapping=slots, block_tables=self.block_tables, ctx_lens=self.ctx_lens,
                        num_splits=self.splits, workspace=self.ws, groups=self.groups, local_logits=self.dist_greedy)
        if hidden is not None:
            logits = e.model.forward(self.input_ids, self.positions, e.kv, meta, hidden=hidden)
        else:
            logits = e.model.forward(self.input_ids, self.positions, e.kv, meta)
        if fused and not self.dist_greedy:
            # ONE launch: K6 sampling + record / advance + the next step's slots, offsets, embeddings
            ops.sample_advance(logits.contiguous(), self.temp, self.top_p, self.top_k, self.seeds, offsets,
                               self.sample_ws, self.nxt, self.out, self.input_ids, self.positions, self.ctx_lens,
                               self.step, self.slots, self.hidden, self.block_tables, e.model.w["embed"], self.bs)
            return
        if self.dist_greedy:
            nxt = e.tp.greedy_gather(logits, e.cfg.vocab)
        else:
            nxt = ops.sample(logits.contiguous(), self.temp, self.top_p, self.top_k, self.seeds, offsets,
                             ws=self.sample_ws)
        # one epilogue launch: record ids, advance positions / lengths / step (+ next step's prep)
        if fused:
            ops.decode_advance(self.out, self.input_ids, self.positions, self.ctx_lens, self.step, nxt,
                               prep=(self.slots, self.offsets, self.hidden, self.block_tables,
                                     e.model.w["embed"], self.bs))
        else:
            ops.decode_advance(self.out, self.input_ids, self.positions, self.ctx_lens, self.step, nxt)

    def _host_buffer(self, k: int) -> torch.Tensor:
        """Pinned [MAX_STEPS, B] int64 copy targets of the sampled ids (two, alternating)."""
        while len(self._host_out) < 2:
            self._host_out.append(torch.empty(MAX_STEPS, self.B, dtype=torch.int64, pin_memory=True))
        return self._host_out[k]

    def check_guard(self) -> None:
        code = int(self.guard_err.item())
        if code:
            self.guard_err.zero_()
            raise AssertionError(f"paging guard tripped in the decode graph (code {code}): "
                                 f"{ops.paging_guard_message(code)}")

    def _reset_groups(self):
        if self.groups is not None:
            self.groups.copy_(torch.tensor([[b, 1, 0] for b in range(self.B)], dtype=torch.int32))

    def _reset_dummy(self):
        self._reset_groups()
        self.positions.zero_()
        self.ctx_lens.fill_(1)
        self.step.zero_()
        self.block_tables.fill_(self.scratch)

    def _capture(self):
        dev = self.engine.device
        self.guard_err.zero_()
        self._reset_dummy()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s), torch.no_grad():
            self._prep()    # slots point into the scratch block, never a live sequence's
            for _ in range(2):  # warm up kernels / allocator / hipBLASLt heuristics outside capture
                self._body()
        torch.cuda.current_stream(dev).wait_stream(s)
        self._reset_dummy()
        with torch.no_grad():
            self._prep()
        # Python's cyclic GC must not run inside the capture: collecting an unreachable engine or
        # graph there frees device memory / destroys a hipGraph while the stream is capturing,
        # which aborts the process (seen when a test's earlier engine was collected mid-capture).
        # The collector switch is process-wide and engines capture from their own threads
        # (orchestrator.execute_plan), so it is reference-counted: off while ANY capture runs.
        with no_gc_during_capture():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), torch.no_grad():
                self._body()
        self.graph = g
        self._reset_dummy()

    def run(self, engine, seqs: Sequence, turns: Sequence, first: torch.Tensor, steps: int, deadline: float,
            eos: int, groups=None) -> List[List[int]]:
        from .engine import _finished
        B = len(seqs)
        dev = engine.device
        steps = min(steps, MAX_STEPS)
        self._reset_dummy()
        bt = torch.full((self.B, self.maxb), self.scratch, dtype=torch.int32)
        for j, s in enumerate(seqs):
            bt[j, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
        if engine.debug_checks:
            engine.check_paging(bt, [])
        self.block_tables.copy_(bt.to(dev, non_blocking=True))
        if self.groups is not None and groups is not None:
            self.groups.copy_(engine.group_table(groups, self.B).to(dev, non_blocking=True))
        lens = torch.tensor([s.length for s in seqs] + [0] * (self.B - B), dtype=torch.int64)
        self.positions.copy_(lens.to(dev, non_blocking=True))
        self.ctx_lens.copy_((lens + 1).to(torch.int32).to(dev, non_blocking=True))
        pad = self.B - B
        self.input_ids.zero_()
        self.input_ids[:B].copy_(first[:B])
        self.temp.copy_(torch.tensor([t.params.temperature for t in turns] + [0.0] * pad, dtype=torch.float32))
        self.top_p.copy_(torch.tensor([t.params.top_p for t in turns] + [1.0] * pad, dtype=torch.float32))
        self.top_k.copy_(torch.tensor([t.params.top_k for t in turns] + [0] * pad, dtype=torch.int32))
        self.seeds.copy_(torch.tensor([t.params.seq_seed(t.seq_key) for t in turns] + [0] * pad, dtype=torch.int64))
        with torch.no_grad():
            self._prep()
        need_tokens = any((not t.params.ignore_eos) or t.params.stop_on_consensus for t in turns)
        # stop checks are pipelined: at every `chunk`-th replay the sampled ids so far are copied
        # to pinned host memory behind an event, and the host inspects the PREVIOUS copy while
        # the GPU keeps replaying — the queue never drains for a check (a synchronous read
        # idled the GPU for the tokenizer decode of every reply, ~1 ms per check). A stop is
        # seen at most 2 chunks (= sync_every) late, as before; extra replays past it are
        # discarded (their K/V lies beyond the kept tokens and is truncated).
        chunk = max(1, engine.ecfg.sync_every // 2) if need_tokens else engine.ecfg.sync_every
        first_host = first[:B].tolist()
        done_at = steps
        pending = None
        replays = engine.stats.get("graph_replays", 0)
        for i in range(1, steps):
            self.graph.replay()
            replays += 1
            engine.stats["graph_replays"] = replays
            if i % chunk == 0:
                if engine.debug_checks:
                    self.check_guard()
                if engine.past_deadline(deadline, i // chunk):
                    engine._sync()
                    raise EngineTimeout("engine", "turn exceeded timeout_per_turn_seconds")
                if need_tokens:
                    host = self._host_buffer((i // chunk) % 2)
                    host[:i].copy_(self.out[:i], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                    prev, pending = pending, (i, host, ev)
                    if prev is not None:
                        j, hbuf, pev = prev
                        pev.synchronize()
                        got = hbuf[:j, :B].t().tolist()
                        outs = [[f] + g for f, g in zip(first_host, got)]
                        if all(_finished(o, t.params, eos, engine.tokenizer) for o, t in zip(outs, turns)):
                            done_at = j + 1
                            break
        if engine.debug_checks:
            self.check_guard()
        n = done_at - 1
        # the same ids kept on the device, [B, n + 1] (C1 all-gathers them without host staging);
        # a copy: the next turn's replays overwrite ``out``
        self.last_dev = torch.cat([first[:B].view(1, B), self.out[:n, :B]], 0).t().contiguous()
        got = self.out[:n, :B].t().tolist() if n > 0 else [[] for _ in range(B)]
        return [[f] + g for f, g in zip(first_host, got)]
