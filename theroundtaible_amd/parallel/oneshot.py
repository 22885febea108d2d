"""K9: one-shot all-reduce for tensor-parallel decode (csrc/oneshot_ar.hip).

Decode all-reduces are latency-bound (``[B, hidden]`` bf16, 16 KB at B = 1 on Llama-3-70B, two
per layer). On an MI355X node every GPU has a dedicated xGMI link to each peer, so instead of
RCCL's ring (world-1 dependent steps) each rank pushes its partial into every peer's IPC-mapped
receive buffer in one step and sums the copies locally. Larger messages (prefill) stay on RCCL.

Set-up is collective over the TP group: each rank allocates uncached receive/flag buffers,
the 128-byte IPC handles are exchanged with ``all_gather_object``, and every rank maps its
peers'. The launch itself is hipGraph-capturable (device-side call counter).
``ROUNDTABLE_ONESHOT_AR=0`` disables it (RCCL everywhere).

Fused form (:meth:`OneShotAllReduce.gemm_ar`): the row-parallel decode GEMMs (o / down) run the
exchange in their own epilogue, tile by tile (skinny_core.h ``EPI_AR``), bit-identical to GEMM +
K9 and with no all-reduce launch. It is used only after :func:`self_test_fused` has compared it
with GEMM + K9 on this node's links; ``ROUNDTABLE_FUSED_AR=0`` keeps the separate launches.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

DEFAULT_CAP_ELEMS = 16 * 8192     # M <= 16 decode rows x hidden 8192 (Llama-3-70B)


def enabled_by_env() -> bool:
    return os.environ.get("ROUNDTABLE_ONESHOT_AR", "1") != "0"


def fused_enabled_by_env() -> bool:
    return os.environ.get("ROUNDTABLE_FUSED_AR", "1") != "0"


class OneShotAllReduce:
    """Use :func:`try_create` (collective); the constructor wraps an already-opened comm."""

    def __init__(self, nat, comm_id: int, rank: int, world: int, cap_elems: int):
        self._nat, self.id = nat, comm_id
        self.world, self.rank, self.cap = world, rank, cap_elems
        self.latency_us: Optional[float] = None   # measured at creation (probe_latency)
        self.fused = False                         # gemm_ar passed its self-test on every rank
        self.fused_saving_us: Optional[float] = None

    def accepts_gemm(self, x: torch.Tensor, Ws: torch.Tensor) -> bool:
        """The fused row-parallel GEMM + all-reduce takes this decode shape."""
        if not (self.fused and self.id is not None and x.is_cuda and x.dim() == 2 and Ws.dim() == 2):
            return False
        M, K = x.shape
        N = Ws.shape[0]
        return (x.dtype == torch.bfloat16 and x.is_contiguous() and 1 <= M <= 16 and K % 32 == 0
                and N % 16 == 0 and N // 16 <= 1024 and M * N <= self.cap and Ws.shape[1] == K)

    def gemm_ar(self, x: torch.Tensor, Ws: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``sum over ranks of x_r @ W_r^T`` ([M, N] bf16) with ``Ws`` = this rank's shuffled
        row-parallel shard: one launch, the K9 exchange in the epilogue."""
        if out is None:
            out = torch.empty(x.shape[0], Ws.shape[0], dtype=x.dtype, device=x.device)
        self._nat.oneshot_gemm_ar(self.id, out, x, Ws)
        return out

    def accepts(self, x: torch.Tensor) -> bool:
        return (self.id is not None and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and 0 < x.numel() <= self.cap and x.data_ptr() % 16 == 0)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        self._nat.oneshot_allreduce(self.id, x)
        return x

    def error(self) -> int:
        """1 if a peer's flag never arrived within the poll bound (that call's result is wrong)."""
        return int(self._nat.oneshot_error(self.id))

    def clear_error(self) -> None:
        self._nat.oneshot_clear_error(self.id)

    def set_poll_limit(self, limit: int) -> None:
        """Flag-wait bound in poll iterations (default ~2^26; fault-injection tests use a tiny one)."""
        if self._nat.oneshot_set_poll_limit(self.id, int(limit)) != 0:
            raise ValueError(f"bad poll limit {limit}")

    def close(self) -> None:
        if self.id is not None:
            self._nat.oneshot_destroy(self.id)
            self.id = None


def try_create(group, rank: int, world: int, cap_elems: int = DEFAULT_CAP_ELEMS) -> Optional[OneShotAllReduce]:
    """Collective over ``group``: the one-shot all-reduce if every rank can build it, else None
    (RCCL path). Two agreement rounds (allocate+export, then map peers) so a rank that fails
    never leaves its peers inside a different collective."""
    from .. import ops
    comm_id, handles, nat = None, None, None
    try:
        nat = ops.native()
        comm_id, handles = nat.oneshot_create(world, rank, cap_elems)
    except Exception:  # noqa: BLE001 - no extension / no IPC on this node
        handles = None
    gathered = [None] * world
    dist.all_gather_object(gathered, handles, group=group)
    ok = 0
    if all(h is not None for h in gathered):
        try:
            nat.oneshot_open(comm_id, b"".join(gathered), world)
            ok = 1
        except Exception:  # noqa: BLE001 - peer mapping refused: RCCL path
            ok = 0
    oks = [None] * world
    dist.all_gather_object(oks, ok, group=group)
    if not all(oks):
        if comm_id is not None:
            nat.oneshot_destroy(comm_id)
        return None
    comm = OneShotAllReduce(nat, comm_id, rank, world, cap_elems)
    # a mapping that opened is not yet a mapping that works: prove the push / flag protocol on
    # THIS node's links (both slots, every rank's values) before any decode depends on it, and
    # agree on the verdict — a single failing rank sends the whole group to RCCL
    passed = self_test(comm)
    verdicts = [None] * world
    dist.all_gather_object(verdicts, passed, group=group)
    if not all(verdicts):
        comm.close()
        return None
    comm.latency_us = probe_latency(comm, group)
    if fused_enabled_by_env():
        passed = self_test_fused(comm)
        verdicts = [None] * world
        dist.all_gather_object(verdicts, passed, group=group)
        comm.fused = all(verdicts)
        if comm.fused:
            comm.fused_saving_us = probe_fused_saving(comm, group)
    return comm


SELF_TEST_POLL_LIMIT = 1 << 20      # ~1 s of flag polling: a dead link fails fast, not in minutes


def self_test(comm: OneShotAllReduce) -> bool:
    """Four calls (both buffer slots twice) of rank-dependent values, checked exactly against
    the host sum, with a short flag-wait bound. Every rank runs the same calls (collective)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    ok = True
    try:
        comm.set_poll_limit(SELF_TEST_POLL_LIMIT)
        n = min(comm.cap, 8 * 2048 * 4)          # several workgroups' slices
        idx = torch.arange(n, device=dev, dtype=torch.float32)
        for call in range(4):
            # small integers: exact in bf16 and in the fp32 sum whatever the rank count
            vals = [((idx + 3 * r + call) % 7) - 3 for r in range(comm.world)]
            x = vals[comm.rank].to(torch.bfloat16).contiguous()
            comm(x)
            want = torch.stack(vals).sum(0)
            torch.cuda.synchronize(dev)
            ok = ok and bool(torch.equal(x.float(), want))
        ok = ok and comm.error() == 0
    except Exception:  # noqa: BLE001 - a launch failure is a failed self-test
        ok = False
    finally:
        try:
            comm.clear_error()
            comm.set_poll_limit(1 << 26)
        except Exception:  # noqa: BLE001
            ok = False
    return ok


def probe_latency(comm: OneShotAllReduce, group, iters: int = 50) -> float:
    """Mean µs per decode-size call (3 rows x 4096, the bench's shape) over ``iters`` back-to-back
    launches, max over ranks: the measured K9 latency the cost model (parallel/costmodel.py)
    otherwise has to assume. Collective."""
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.zeros(3 * 4096, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        comm(x)
    torch.cuda.synchronize(dev)
    _group_max(torch.zeros(1, dtype=torch.float64), group, dev)      # line the ranks up
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        comm(x)
    e.record()
    torch.cuda.synchronize(dev)
    us = s.elapsed_time(e) * 1e3 / iters
    return round(_group_max(torch.tensor([us], dtype=torch.float64), group, dev), 2)


def _group_max(t: torch.Tensor, group, dev) -> float:
    if dist.get_backend(group) != "gloo":
        t = t.to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def _fused_case(comm: OneShotAllReduce, M: int, N: int, K: int, seed: int):
    from .. import ops
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator().manual_seed(seed + 7919 * comm.rank)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(dev)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    return x, ops.shuffle_weight(W)


def self_test_fused(comm: OneShotAllReduce) -> bool:
    """The fused GEMM + exchange against the separate GEMM + K9 launches on the same inputs:
    bit-identical on every rank, no flag-wait expiry, across both buffer slots and interleaved
    with K9 calls (they share the comm's call counter). Collective."""
    from .. import ops
    dev = torch.device("cuda", torch.cuda.current_device())
    ok = True
    try:
        comm.set_poll_limit(SELF_TEST_POLL_LIMIT)
        comm.fused = True                                    # accepts_gemm() needs it
        for i, (M, N, K) in enumerate([(3, 4096, 512), (1, 4096, 1792), (5, 8192, 1024)]):
            if M * N > comm.cap:
                continue
            x, Ws = _fused_case(comm, M, N, K, 100 + i)
            want = ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_STORE)
            comm(want)                                       # separate K9 launch
            for _ in range(2):                               # both slots
                got = comm.gemm_ar(x, Ws)
                torch.cuda.synchronize(dev)
                ok = ok and bool(torch.equal(got, want))
        ok = ok and comm.error() == 0
    except Exception:  # noqa: BLE001 - a launch failure is a failed self-test
        ok = False
    finally:
        comm.fused = False
        try:
            comm.clear_error()
            comm.set_poll_limit(1 << 26)
        except Exception:  # noqa: BLE001
            ok = False
    return ok


def probe_fused_saving(comm: OneShotAllReduce, group, iters: int = 50) -> float:
    """µs saved per row-parallel GEMM by the fused form vs GEMM + K9 at the bench's o-projection
    shard shape (M = 3, N = 4096, K = 4096 / world), max over ranks. Collective."""
    from .. import ops
    dev = torch.device("cuda", torch.cuda.current_device())
    x, Ws = _fused_case(comm, 3, 4096, max(32, 4096 // comm.world), 300)
    out = torch.empty(3, 4096, dtype=torch.bfloat16, device=dev)

    def timed(fn) -> float:
        for _ in range(5):
            fn()
        torch.cuda.synchronize(dev)
        _group_max(torch.zeros(1, dtype=torch.float64), group, dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize(dev)
        return _group_max(torch.tensor([s.elapsed_time(e) * 1e3 / iters], dtype=torch.float64), group, dev)

    sep = timed(lambda: comm(ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_STORE)))
    fused = timed(lambda: comm.gemm_ar(x, Ws, out))
    return round(sep - fused, 2)
