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
with GEMM + K9 on this node's links, and by default only when every rank owns its GPU
(:func:`fused_mode_env`) and when a timed probe on the node shows it beating GEMM + K9 (on one
GPU shared by two rehearsal ranks it loses by ~46 µs: the two processes' spinning grids
co-schedule badly); ``ROUNDTABLE_FUSED_AR=0`` keeps the separate launches.

LL protocol (:func:`choose_protocol`): the all-reduce (standalone launch AND the fused EPI_AR
epilogue) can carry the call's epoch in every 8-byte store next to the data, so receivers poll the
data itself — no system fence (an xGMI round trip) and no separate flag. Chosen per node by an
exact self-test and a timed probe; the gather keeps flags.

Epoch agreement (:meth:`OneShotAllReduce.resync`): the call counter is device-local, so ranks that
issued different numbers of calls (one rank's capture warm-up failed part-way, an abandoned turn)
would wait on epochs their peers never write. The engine re-agrees it (group MAX, buffers zeroed)
whenever the group recovers, falls back from a failed capture, or fails a turn on an expired wait.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

DEFAULT_CAP_ELEMS = 16 * 8192     # M <= 16 decode rows x hidden 8192 (Llama-3-70B)


def enabled_by_env() -> bool:
    return os.environ.get("ROUNDTABLE_ONESHOT_AR", "1") != "0"


def fused_mode_env() -> str:
    """``ROUNDTABLE_FUSED_AR``: ``auto`` (default: only when every rank owns its GPU and the timed
    probe shows a saving), ``probe`` (self-test + timed decision even on a shared GPU — exercises
    the auto decision in rehearsals), ``1`` (forced, also on a shared GPU: the 2-rank numerics
    rehearsal), ``0`` (never)."""
    return os.environ.get("ROUNDTABLE_FUSED_AR", "auto")


def ll_mode_env() -> str:
    """``ROUNDTABLE_K9_LL``: protocol of the standalone all-reduce launch. ``auto`` (default): the
    LL form (data + epoch in one 8-byte store, no fence) after its exact self-test, when the timed
    probe on this node's links shows it faster than push + fence + flag; ``1``: LL after a passing
    self-test; ``0``: push + fence + flag only."""
    return os.environ.get("ROUNDTABLE_K9_LL", "auto")


def _device_key() -> str:
    """Physical identity of this rank's GPU (PCI location when exposed, else UUID, else index)."""
    import socket
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    pci = tuple(getattr(props, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if all(v is not None for v in pci):
        ident = "pci:%s:%s:%s" % pci
    elif getattr(props, "uuid", None) is not None:
        ident = f"uuid:{props.uuid}"
    else:
        ident = f"index:{torch.cuda.current_device()}"
    return f"{socket.gethostname()}/{ident}"


class OneShotAllReduce:
    """Use :func:`try_create` (collective); the constructor wraps an already-opened comm."""

    def __init__(self, nat, comm_id: int, rank: int, world: int, cap_elems: int):
        self._nat, self.id = nat, comm_id
        self.world, self.rank, self.cap = world, rank, cap_elems
        self.latency_us: Optional[float] = None   # measured at creation (probe_latency)
        self.fused = False                         # gemm_ar passed its self-test on every rank
        self.fused_saving_us: Optional[float] = None
        self.distinct_gpus = False                  # every rank of the group on its own device
        self.gather_ok = False                      # one-shot all-gather passed its self-test
        self.gather_saving_us: Optional[float] = None
        self.ll = False                             # standalone all-reduce in the LL form
        self.flag_latency_us: Optional[float] = None
        self.ll_latency_us: Optional[float] = None

    group = None                                    # the TP process group (set by try_create)
    resyncs = 0

    def epoch(self) -> int:
        """This rank's device call counter (host read; synchronises the device)."""
        e = int(self._nat.oneshot_epoch(self.id))
        if e < 0:
            raise RuntimeError(f"oneshot_epoch failed (rc={e})")
        return e

    def resync(self) -> bool:
        """Collective over the TP group: re-agree the call counter after ranks may have issued
        different numbers of K9 calls (a capture warm-up that failed part-way on one rank, a turn
        abandoned mid-decode, an injected extra call). Every rank quiesces its device, the group
        takes the MAX of the ranks' epochs (one all-reduce, which is also the first barrier), each
        rank sets its counter to it and zeroes every receive buffer it owns (flags, tile flags,
        gather flags, LL pairs: no stale tag can match a future epoch), and a second all-reduce —
        the barrier before any rank's next call can push into a peer's buffer — agrees that every
        rank succeeded. Returns False (on every rank) if any rank failed: the caller drops K9."""
        dev = torch.device("cuda", torch.cuda.current_device())
        rc = 0
        try:
            torch.cuda.synchronize(dev)
            e = self.epoch()
        except Exception:  # noqa: BLE001 - a dead device: the group drops K9 together
            e, rc = 0, 1
        E = int(_group_max(torch.tensor([float(e)], dtype=torch.float64), self.group, dev))
        if rc == 0:
            try:
                rc = 0 if int(self._nat.oneshot_resync(self.id, E)) == 0 else 1
            except Exception:  # noqa: BLE001
                rc = 1
        ok = _group_max(torch.tensor([float(rc)], dtype=torch.float64), self.group, dev) == 0
        self.resyncs += 1
        return ok

    def set_ll(self, on: bool) -> None:
        if self._nat.oneshot_set_ll(self.id, bool(on)) != 0:
            raise RuntimeError("oneshot_set_ll failed")
        self.ll = bool(on)

    def accepts_gemm(self, x: torch.Tensor, Ws: torch.Tensor) -> bool:
        """The fused row-parallel GEMM + all-reduce takes this decode shape."""
        if not (self.fused and self.id is not None and x.is_cuda and x.dim() == 2 and Ws.dim() == 2):
            return False
        M, K = x.shape
        N = Ws.shape[0]
        return (x.dtype == torch.bfloat16 and x.is_contiguous() and 1 <= M <= 16 and K % 32 == 0
                and N % 16 == 0 and N // 16 <= 1024 and M * N <= self.cap and Ws.shape[1] == K)

    def accepts_gather(self, x: torch.Tensor) -> bool:
        """The one-shot all-gather takes this [rows, shard] slice (C3 logits)."""
        if not (self.gather_ok and self.id is not None and x.is_cuda and x.dim() == 2):
            return False
        rows, shard = x.shape
        return (x.dtype == torch.bfloat16 and x.is_contiguous() and shard % 8 == 0
                and rows * shard * self.world <= self._nat.oneshot_gather_capacity())

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        """[rows, shard] per rank -> [rows, world * shard] in rank order, one launch."""
        out = torch.empty(x.shape[0], x.shape[1] * self.world, dtype=x.dtype, device=x.device)
        self._nat.oneshot_allgather(self.id, _aligned(x), out, self.world)
        return out

    def gemm_ar(self, x: torch.Tensor, Ws: torch.Tensor, out: Optional[torch.Tensor] = None,
                res: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``sum over ranks of x_r @ W_r^T`` ([M, N] bf16) with ``Ws`` = this rank's shuffled
        row-parallel shard: one launch, the K9 exchange in the epilogue. ``res``: the residual
        form — ``res = bf16(res + bf16(sum))`` in place (returned), nothing else written."""
        if res is not None:
            if res.data_ptr() % 16 == 0 and res.is_contiguous():
                self._nat.oneshot_gemm_ar(self.id, res, _aligned(x), Ws, res)
                return res
            # (rank-invariant collective either way: the same fused call, then a local add)
            return res.add_(self.gemm_ar(x, Ws, out))
        if out is None:
            out = torch.empty(x.shape[0], Ws.shape[0], dtype=x.dtype, device=x.device)
        self._nat.oneshot_gemm_ar(self.id, out, _aligned(x), Ws)
        return out

    def accepts(self, x: torch.Tensor) -> bool:
        # rank-invariant conditions only (shape, dtype, layout): every rank of the group must take
        # the same path, so a rank-dependent property such as the address alignment is handled
        # by staging (__call__), never by falling back on one rank alone
        return (self.id is not None and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and 0 < x.numel() <= self.cap)

    def __call__(self, x: torch.Tensor, res: Optional[torch.Tensor] = None) -> torch.Tensor:
        """In-place sum over the group; with ``res``: ``res = bf16(res + bf16(sum))`` in place
        (the residual form, ``x`` left as it was), returns ``res``."""
        if res is not None:
            if x.data_ptr() % 16 == 0 and res.data_ptr() % 16 == 0 and res.is_contiguous():
                self._nat.oneshot_allreduce(self.id, x, res)
                return res
            return res.add_(self(x))      # same single K9 call on every rank, then a local add
        if x.data_ptr() % 16:
            t = x.clone()                 # fresh allocations are 16-B aligned
            self._nat.oneshot_allreduce(self.id, t)
            x.copy_(t)
            return x
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


def _aligned(x: torch.Tensor) -> torch.Tensor:
    """``x`` itself when 16-B aligned (the kernels' vector loads), else an aligned copy."""
    return x if x.data_ptr() % 16 == 0 else x.clone()


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
    comm.group = group
    # a mapping that opened is not yet a mapping that works: prove the push / flag protocol on
    # THIS node's links (both slots, every rank's values) before any decode depends on it, and
    # agree on the verdict — a single failing rank sends the whole group to RCCL
    passed = self_test(comm)
    verdicts = [None] * world
    dist.all_gather_object(verdicts, passed, group=group)
    if not all(verdicts):
        comm.close()
        return None
    comm.latency_us = comm.flag_latency_us = probe_latency(comm, group)
    choose_protocol(comm, group)
    passed = self_test_gather(comm)
    verdicts = [None] * world
    dist.all_gather_object(verdicts, passed, group=group)
    comm.gather_ok = all(verdicts)
    # The fused form keeps a whole GEMM grid spinning on its peers' tiles. With one rank per GPU
    # every workgroup is resident (<= 2 tiles per CU at decode shapes), so the wait always ends.
    # Ranks SHARING a GPU (rehearsals) additionally need the other processes' kernels to be
    # scheduled while those grids spin, which the hardware queue scheduler does not promise beyond
    # two processes (a 4-rank rehearsal timed out) — there the separate K9 launch stays the default.
    keys = [None] * world
    dist.all_gather_object(keys, _device_key(), group=group)
    comm.distinct_gpus = len(set(keys)) == world
    mode = fused_mode_env()
    if mode in ("1", "probe") or (mode == "auto" and comm.distinct_gpus):
        passed = self_test_fused(comm)
        verdicts = [None] * world
        dist.all_gather_object(verdicts, passed, group=group)
        if all(verdicts):
            # measure, don't guess: the fused form must beat GEMM + K9 on THIS node's links (the
            # saving is the group max of each form's time, so every rank takes the same decision)
            comm.fused_saving_us = probe_fused_saving(comm, group)
            expired = _group_max(torch.tensor([float(comm.error())], dtype=torch.float64), group,
                                 torch.device("cuda", torch.cuda.current_device())) > 0
            comm.clear_error()
            comm.fused = mode == "1" or (not expired and comm.fused_saving_us >= MIN_FUSED_SAVING_US)
    if comm.gather_ok and dist.get_backend(group) != "gloo":
        # the one-shot gather replaces an RCCL all-gather: keep whichever this node runs faster
        comm.gather_saving_us = probe_gather_saving(comm, group)
        comm.gather_ok = comm.gather_saving_us > 0.0
    lim = os.environ.get("ROUNDTABLE_K9_POLL_LIMIT")
    if lim:          # tests: a short flag-wait bound so an injected desync expires in ms, not s
        comm.set_poll_limit(int(lim))
    return comm


MIN_FUSED_SAVING_US = 0.5          # per call, at the o-projection shard shape
MIN_LL_SAVING_US = 0.2             # per call, at the bench's all-reduce shape


def choose_protocol(comm: OneShotAllReduce, group) -> None:
    """Collective: the LL form replaces push + fence + flag for the standalone all-reduce when it
    passes the same exact self-test on every rank and (``auto``) its group-max latency beats the
    flag form's by ``MIN_LL_SAVING_US`` — identical numbers, so every rank takes the same
    decision. The fused GEMM form (EPI_AR epilogue) follows the same choice — ``oneshot_gemm_ar``
    passes the comm's protocol to the epilogue, and the fused self-test / saving probe run after
    this, on the chosen form; only the one-shot gather keeps the flag protocol."""
    mode = ll_mode_env()
    if mode == "0":
        return
    comm.set_ll(True)
    passed = self_test(comm)
    verdicts = [None] * comm.world
    dist.all_gather_object(verdicts, passed, group=group)
    if not all(verdicts):
        comm.set_ll(False)
        return
    comm.ll_latency_us = probe_latency(comm, group)
    use = mode == "1" or comm.ll_latency_us <= comm.flag_latency_us - MIN_LL_SAVING_US
    comm.set_ll(use)
    comm.latency_us = comm.ll_latency_us if use else comm.flag_latency_us

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


def self_test_gather(comm: OneShotAllReduce) -> bool:
    """The one-shot all-gather against the known concatenation (rank-dependent integers, exact),
    at the bench's logit-slice shape and a small one, both slots. Collective."""
    dev = torch.device("cuda", torch.cuda.current_device())
    ok = True
    try:
        comm.set_poll_limit(SELF_TEST_POLL_LIMIT)
        comm.gather_ok = True
        for i, (rows, shard) in enumerate([(3, 128256 // comm.world), (1, 64), (2, 4096)]):
            shard -= shard % 8
            if not comm.accepts_gather(torch.empty(rows, shard, dtype=torch.bfloat16, device=dev)):
                continue
            cols = torch.arange(rows * shard, device=dev, dtype=torch.float32).view(rows, shard)
            parts = [((cols + 5 * r + i) % 11) - 5 for r in range(comm.world)]
            got = comm.all_gather_last(parts[comm.rank].to(torch.bfloat16).contiguous())
            torch.cuda.synchronize(dev)
            ok = ok and bool(torch.equal(got.float(), torch.cat(parts, dim=1)))
        ok = ok and comm.error() == 0
    except Exception:  # noqa: BLE001 - a launch failure is a failed self-test
        ok = False
    finally:
        comm.gather_ok = False
        try:
            comm.clear_error()
            comm.set_poll_limit(1 << 26)
        except Exception:  # noqa: BLE001
            ok = False
    return ok


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


def _timed_us(fn, group, dev, iters: int = 50) -> float:
    """Mean µs per call of ``fn`` over ``iters`` back-to-back launches, max over the group."""
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


def probe_gather_saving(comm: OneShotAllReduce, group) -> float:
    """µs saved per C3 logits gather ([3, 128256 / world] bf16) by the one-shot all-gather vs the
    process group's all-gather into [world, 3, shard] + the permute to [3, world * shard]."""
    dev = torch.device("cuda", torch.cuda.current_device())
    shard = (128256 // comm.world) // 8 * 8
    x = torch.zeros(3, shard, dtype=torch.bfloat16, device=dev)
    flat = torch.empty(comm.world * 3, shard, dtype=torch.bfloat16, device=dev)

    def rccl():
        dist.all_gather_into_tensor(flat, x, group=group)
        flat.view(comm.world, 3, shard).movedim(0, -2).reshape(3, comm.world * shard)

    return round(_timed_us(rccl, group, dev) - _timed_us(lambda: comm.all_gather_last(x), group, dev), 2)


def probe_fused_saving(comm: OneShotAllReduce, group, iters: int = 50) -> float:
    """µs saved per row-parallel GEMM by the fused form vs GEMM + K9 at the bench's o-projection
    shard shape (M = 3, N = 4096, K = 4096 / world), max over ranks. Collective."""
    from .. import ops
    dev = torch.device("cuda", torch.cuda.current_device())
    x, Ws = _fused_case(comm, 3, 4096, max(32, 4096 // comm.world), 300)
    out = torch.empty(3, 4096, dtype=torch.bfloat16, device=dev)
    sep = _timed_us(lambda: comm(ops.skinny_gemm(x, Ws, ops.PRO_PLAIN, ops.EPI_STORE)), group, dev, iters)
    fused = _timed_us(lambda: comm.gemm_ar(x, Ws, out), group, dev, iters)
    return round(sep - fused, 2)
