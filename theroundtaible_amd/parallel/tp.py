"""Tensor parallelism (Megatron-style) for oversized knights.

Column-parallel: fused QKV (whole heads per rank) and gate/up; row-parallel: o_proj
and down_proj followed by one RCCL all-reduce each (C2); the lm_head is
vocab-parallel followed by an all-gather of the logit shards (C3). One process per
GPU; ``torch.distributed`` backend ``nccl`` is RCCL on ROCm, ``gloo`` on CPU tests.

Decode all-reduces are tiny (``[B, hidden]`` bf16 = 16 KB at B=1, 70B): they are
latency-bound on xGMI, so they are issued on the compute stream inside the captured
hipGraph rather than bucketed, and go through the one-shot IPC all-reduce (K9,
``parallel/oneshot.py``: one push step over the dedicated xGMI links instead of a ring)
when every rank could map its peers; larger messages (prefill) use RCCL.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class TPInfo:
    size: int = 1
    rank: int = 0
    group: Optional[object] = None   # torch.distributed ProcessGroup
    oneshot: Optional[object] = None  # parallel.oneshot.OneShotAllReduce (decode-size messages)
    # gloo group over the same ranks with the engine-load timeout (parallel/cluster.py
    # load_group_for): Engine construction meets there after loading its weights and before the
    # group's first collective (K9 set-up), so a rank that loads slowly is waited for with the load
    # limit, not the short containment timeout of ``group``
    load_group: Optional[object] = None

    @property
    def enabled(self) -> bool:
        return self.size > 1

    def shard(self, n: int) -> int:
        if n % self.size:
            raise ValueError(f"dimension {n} not divisible by tp={self.size}")
        return n // self.size

    def backend(self) -> str:
        return dist.get_backend(self.group) if self.size > 1 else "none"

    def kv_heads(self, n_kv: int) -> int:
        """KV heads held per rank: an even split, or ONE (replicated) when the group is wider
        than the model's KV heads — ranks ``r`` with equal ``r * n_kv // size`` share a head
        (GQA: their query heads all read it). Needs ``size % n_kv == 0`` then."""
        if n_kv >= self.size:
            return self.shard(n_kv)
        if self.size % n_kv:
            raise ValueError(f"tp={self.size} is neither a divisor nor a multiple of the {n_kv} KV heads")
        return 1

    def kv_head0(self, n_kv: int) -> int:
        """First (global) KV head of this rank's shard."""
        return self.rank * n_kv // self.size if n_kv < self.size else self.rank * self.shard(n_kv)

    def _host_staged(self, x: torch.Tensor) -> bool:
        # gloo (CPU CI, or the shared-GPU rehearsal mode of parallel/cluster.py) moves GPU
        # tensors through host memory explicitly; RCCL works on device memory directly
        return x.is_cuda and self.backend() == "gloo"

    def setup_oneshot(self) -> None:
        """Collective over the group (every rank calls it at the same point)."""
        from .oneshot import enabled_by_env, try_create
        if self.size > 1 and self.oneshot is None and enabled_by_env():
            self.oneshot = try_create(self.group, self.rank, self.size)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.oneshot is not None and self.oneshot.accepts(x):
                return self.oneshot(x)
            if self._host_staged(x):
                h = x.cpu()
                dist.all_reduce(h, group=self.group)
                x.copy_(h)
            else:
                dist.all_reduce(x, group=self.group)
        return x

    def all_reduce_into(self, x: torch.Tensor, res: torch.Tensor) -> torch.Tensor:
        """C2 with the residual add fused: ``res = bf16(res + bf16(sum over ranks of x))`` in
        place (K9's residual form; host collectives + a bf16 add otherwise, the same bits)."""
        if self.size > 1 and self.oneshot is not None and self.oneshot.accepts(x):
            return self.oneshot(x, res=res)
        return res.add_(self.all_reduce(x))

    def row_parallel(self, x: torch.Tensor, Ws: torch.Tensor, res: Optional[torch.Tensor] = None,
                     **gemm_kw) -> torch.Tensor:
        """Decode row-parallel linear (o / down on shuffled weights) + C2: ONE launch with the
        K9 exchange fused into the GEMM epilogue when the one-shot comm passed its fused self-test,
        else the skinny GEMM followed by :meth:`all_reduce`. ``res``: the decode residual stream —
        the all-reduced output is added into it in place (the same epilogue / K9 launch), so the
        next GEMM reads it with a plain RMSNorm prologue, exactly as at tp 1."""
        from .. import ops
        os_ = self.oneshot
        if self.size > 1 and os_ is not None and os_.accepts_gemm(x, Ws):
            self.fused_ar_calls = getattr(self, "fused_ar_calls", 0) + 1
            return os_.gemm_ar(x, Ws, res=res)
        y = ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_STORE, **gemm_kw)
        return self.all_reduce(y) if res is None else self.all_reduce_into(y, res)

    def any_rank(self, flag: bool) -> bool:
        """True if ``flag`` is set on any rank of the group (host-side agreement, e.g. to fail a
        turn on every rank of a TP knight when one rank's K9 flag wait expired)."""
        if self.size == 1:
            return flag
        return self.group_min(0 if flag else 1) == 0

    def group_min(self, v: int) -> int:
        """The minimum of ``v`` over the group (host-side agreement, one small collective)."""
        if self.size == 1:
            return v
        dev = "cpu" if self.backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([v], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def greedy_gather(self, local: torch.Tensor, vocab: int) -> torch.Tensor:
        """C3 for greedy decoding without moving the logits: every rank takes the argmax of its
        vocab shard, the group all-gathers ``[B, 2]`` (value, global id) and picks the best —
        ``B * 8`` bytes per rank instead of ``B * V/tp * 4``. Ties resolve to the lowest id,
        like an argmax over the gathered row. Returns ``[B]`` int64 ids on ``local``'s device."""
        B, vs = local.shape
        off = self.rank * vs
        lim = max(0, min(vs, vocab - off))        # zero-padded vocab rows never win
        val, idx = local[:, :lim].float().max(dim=1)
        pair = torch.stack([val, (idx + off).float()], dim=1)
        self.c3_greedy_calls = getattr(self, "c3_greedy_calls", 0) + 1
        if self.size == 1:
            return pair[:, 1].long()
        src = pair.cpu() if self._host_staged(local) else pair
        flat = src.new_empty((self.size * B, 2))
        dist.all_gather_into_tensor(flat, src, group=self.group)   # one collective, no per-rank copies
        g = flat.view(self.size, B, 2).to(local.device)    # [tp, B, 2]
        best = g[..., 0].argmax(dim=0)                     # first max = lowest rank = lowest id
        return g[best, torch.arange(B, device=local.device), 1].long()

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        """Concatenate shards along the last dim (vocab-parallel logits).

        Sampled (temperature / top-p) TP decode keeps this gather on purpose: an exact
        distributed nucleus needs the global max, then a mass histogram, then (refinement) a
        second histogram and finally a (value, id) gather — four dependent collectives of a few
        µs latency each on xGMI — while this is ONE all-gather of ``B * V * 4`` bytes (1.5 MB at
        B = 3, Llama-3 vocab: ~10 µs spread over the tp-1 peer links). A Gumbel-argmax "accept"
        shortcut (csrc/sampling.hip) needs a fallback for rejected rows, which a captured graph
        cannot branch into, so it would not remove the gather either. Greedy decode, where one
        (value, id) pair per rank is exact, uses :meth:`greedy_gather`. On GPU groups the gather
        runs as K9's one-shot all-gather (every rank pushes its slice into every peer's buffer,
        csrc/oneshot_ar.hip) once that passed its creation self-test, else over RCCL."""
        if self.size == 1:
            return x
        if self.oneshot is not None and self.oneshot.accepts_gather(x):
            # one launch, one xGMI hop, written straight into [rows, tp * shard] (K9's comm)
            self.oneshot_gathers = getattr(self, "oneshot_gathers", 0) + 1
            return self.oneshot.all_gather_last(x)
        src = x.contiguous().cpu() if self._host_staged(x) else x.contiguous()
        # ONE all-gather into a [tp, rows, shard] buffer and ONE permuting copy (a list-output
        # all_gather + cat costs a copy kernel per rank on top, inside every decode step)
        flat = src.new_empty((self.size * src.shape[0],) + tuple(src.shape[1:]))
        dist.all_gather_into_tensor(flat, src, group=self.group)
        out = flat.view(self.size, *src.shape).movedim(0, -2).reshape(*src.shape[:-1], self.size * src.shape[-1])
        return out.to(x.device)


class SimulatedTP(TPInfo):
    """Cost-model stand-in (``bench.py --simulate-tp N``, tools/tp_cost.py): ONE process computes
    rank 0's shard of a tp=N knight — the exact per-rank GEMM / attention / sampler shapes, in
    the captured decode graph — with every collective replaced by a local op of the same output
    shape. ``comm_us`` set (bench default: K9 5 µs per all-reduce, 9.5 µs per logits gather):
    each collective ALSO launches a device kernel that holds as many CUs as the real K9 launch
    for that long (csrc/oneshot_ar.hip ``sim_comm_spin``), so the simulated step pays its
    communication inside the graph, on the stream, as a node would — and a schedule that hides it
    (:func:`~theroundtaible_amd.models.llama.LlamaModel.forward_decode_fused_tp_mb`) can be
    measured on one GPU. ``comm_us=None``: collectives are free (round-4 compute-only records).
    Never used for a real multi-GPU run."""

    def __init__(self, size: int, comm_us: Optional[float] = None, gather_us: Optional[float] = None):
        super().__init__(size=size, rank=0, group=None)
        self.comm_us = comm_us
        self.gather_us = gather_us if gather_us is not None else comm_us
        self.stand_in_launch_us: Optional[float] = None

    def backend(self) -> str:
        return "nccl"            # keep hipGraph capture on, as on a real RCCL group

    def setup_oneshot(self) -> None:
        self.oneshot = None

    def calibrate_stand_in(self) -> float:
        """What a zero-length spin node costs inside a captured graph, back to back (subtracted,
        so a simulated collective costs ``comm_us`` per call in the captured step, node overhead
        included)."""
        if self.stand_in_launch_us is None:
            from .. import ops
            nat = ops.native()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(8):
                    nat.sim_comm_spin(0, 6)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(100):
                    nat.sim_comm_spin(0, 6)
            g.replay()
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                g.replay()
                b.record()
                torch.cuda.synchronize()
                best = min(best, a.elapsed_time(b) * 1e3 / 100)
            self.stand_in_launch_us = best
        return self.stand_in_launch_us

    def _spin(self, us: Optional[float], numel: int) -> None:
        if not us:
            return
        from .. import ops
        nb = max(1, min(64, numel // 2048))       # the K9 launch's workgroup count for this message
        ticks = int(max(0.0, us - self.calibrate_stand_in()) * 100)   # s_memrealtime: 100 MHz
        ops.native().sim_comm_spin(ticks, nb)
        self.sim_comm_calls = getattr(self, "sim_comm_calls", 0) + 1

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        self.sim_all_reduces = getattr(self, "sim_all_reduces", 0) + 1
        if x.is_cuda:
            self._spin(self.comm_us, x.numel())
        return x

    def row_parallel(self, x: torch.Tensor, Ws: torch.Tensor, res: Optional[torch.Tensor] = None,
                     **gemm_kw) -> torch.Tensor:
        """The shard GEMM, the residual add kept (RESID epilogue: the work K9's residual form does
        besides communicating), then the simulated all-reduce."""
        from .. import ops
        if res is not None:
            self.sim_all_reduces = getattr(self, "sim_all_reduces", 0) + 1
            out = ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_RESID, res=res, **gemm_kw)
            self._spin(self.comm_us, res.numel())
            return out
        return self.all_reduce(ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_STORE, **gemm_kw))

    def any_rank(self, flag: bool) -> bool:
        return flag

    def group_min(self, v: int) -> int:
        return v

    def greedy_gather(self, local: torch.Tensor, vocab: int) -> torch.Tensor:
        lim = max(1, min(local.shape[1], vocab))
        return local[:, :lim].float().argmax(dim=1)

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        out = x.repeat(1, self.size)
        if x.is_cuda:
            self._spin(self.gather_us, out.numel())
        return out


def shard_rows(w: torch.Tensor, tp: TPInfo) -> torch.Tensor:
    """Slice the output (row of [out, in]) dimension: column-parallel linear."""
    n = tp.shard(w.shape[0])
    return w[tp.rank * n:(tp.rank + 1) * n].contiguous()


def shard_cols(w: torch.Tensor, tp: TPInfo) -> torch.Tensor:
    """Slice the input dimension: row-parallel linear."""
    n = tp.shard(w.shape[1])
    return w[:, tp.rank * n:(tp.rank + 1) * n].contiguous()
