"""Process topology: one process per GPU, RCCL world + gloo control plane.

``torch.distributed`` with backend ``nccl`` is RCCL on ROCm; every rank owns exactly
one GPU (``cuda:LOCAL_RANK``). A second, CPU ``gloo`` group carries host control
traffic (seeds, turn metadata, error strings) so tiny Python objects never stall the
xGMI links, and so the whole control plane also runs in CPU-only CI (world_size > 1
with gloo everywhere).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class Cluster:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: str = "cpu"      # this rank's device: cuda:LOCAL_RANK (or shared round-robin in rehearsal mode)
    backend: str = "none"
    cpu_group: Optional[object] = None
    # gloo group with a very long timeout for waits on a PERSON or an idle client (the King's
    # answer, a server's next request): the data and control collectives keep the short,
    # containment-sized timeout of init_cluster
    wait_group: Optional[object] = None
    # gloo group whose timeout covers engine loading (LOAD_TIMEOUT_S): the load rendezvous
    # (load_rendezvous) runs on it, so a rank that loads a checkpoint minutes longer than its
    # peers is waited for there, not in a short-timeout collective
    load_group: Optional[object] = None
    timeout_s: int = 1800        # containment timeout of the world / control (and TP) groups

    def load_rendezvous(self) -> None:
        """Every rank has finished loading its engines (no-op for one rank)."""
        if self.distributed and self.load_group is not None:
            dist.barrier(group=self.load_group)

    @property
    def is_leader(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1

    # ---- control plane (gloo) -------------------------------------------------------------
    def broadcast_object(self, obj: Any, src: int = 0, wait: bool = False) -> Any:
        """``wait``: over :attr:`wait_group` (no containment timeout: rank ``src`` may be waiting
        on a human or an HTTP client)."""
        if not self.distributed:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.wait_group if wait else self.cpu_group)
        return box[0]

    def all_gather_object(self, obj: Any) -> List[Any]:
        if not self.distributed:
            return [obj]
        out: List[Any] = [None] * self.world
        dist.all_gather_object(out, obj, group=self.cpu_group)
        return out

    def barrier(self) -> None:
        if self.distributed or self.backend == "nccl":   # (a 1-rank RCCL world: tools/nccl_check.py)
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def max_scalar(self, x: float) -> float:
        if not self.distributed:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.cpu_group)
        return float(t[0])

    def sum_scalar(self, x: float) -> float:
        if not self.distributed:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.cpu_group)
        return float(t[0])


_CLUSTER: Optional[Cluster] = None


WAIT_TIMEOUT_S = 7 * 24 * 3600
# engine loading: the failsafe guard's per-stage limit (engine_load / k9_create, 900 s) plus margin;
# a rank that really hangs there is ended by the guard first, with the stage named
LOAD_STAGE_LIMIT_S = 900.0
LOAD_TIMEOUT_S = int(LOAD_STAGE_LIMIT_S + 60)


def load_group_for(ranks) -> Optional[object]:
    """A gloo group over ``ranks`` with the load timeout (collective over the WORLD: call it in the
    same order on every rank, like ``dist.new_group``)."""
    if not dist.is_initialized():
        return None
    return dist.new_group(list(ranks), backend="gloo", timeout=datetime.timedelta(seconds=LOAD_TIMEOUT_S))


SHARED_GPU_QUEUE_BUDGET = 16   # hardware queues the ranks sharing one card may map together


def limit_shared_gpu_queues(env: dict, world: int) -> Optional[int]:
    """Rehearsal ranks sharing a card (``ROUNDTABLE_DIST_BACKEND=gloo``, more ranks than GPUs): cap
    each rank's hardware queues (HIP's default is 4) in the launcher's child ``env`` so that all of
    them stay mapped at once. Measured on one MI355X: 8 ranks x 4 queues hung the first captured K9
    warm-up (a one-shot all-reduce whose peers' queues are not mapped waits out its poll bound,
    call after call); 8 x 2 ran the full bench with 0 failed turns (profiles/r05/rehearsal/). The
    HIP runtime reads the variable when it starts, so only a launcher (bench.py, ``roundtable``'s
    SPMD launch) can set it for its ranks; it only ever lowers a value already in ``env`` (the GPU
    boxes export HIP's default, 4). Returns the cap set."""
    if world <= 1 or env.get("ROUNDTABLE_DIST_BACKEND", "").strip().lower() != "gloo":
        return None
    ndev = max(1, torch.cuda.device_count())      # counts devices without starting the runtime
    per_dev = -(-world // ndev)
    try:
        have = int(env.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        have = 4
    q = max(1, SHARED_GPU_QUEUE_BUDGET // per_dev)
    if per_dev * have <= SHARED_GPU_QUEUE_BUDGET or q >= have:
        return None
    env["GPU_MAX_HW_QUEUES"] = str(q)
    return q


def _card_cus(default: int = 256) -> int:
    """Compute units of the first GPU from the KFD topology (no HIP runtime start)."""
    import glob
    for f in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            kv = dict(line.split()[:2] for line in open(f) if len(line.split()) >= 2)
            simd, per = int(kv.get("simd_count", 0)), int(kv.get("simd_per_cu", 0))
        except (OSError, ValueError):
            continue
        if simd > 0 and per > 0:
            return simd // per
    return default


def rehearsal_cu_split(world: int, local: int) -> Optional[str]:
    """``ROUNDTABLE_REHEARSAL_CU_SPLIT=1`` (rehearsal ranks sharing a card): give each rank a
    disjoint slice of the card's CUs (``ROC_GLOBAL_CU_MASK``, read when the HIP runtime starts,
    so this runs first), so the ranks' kernels co-run like kernels on separate GPUs instead of
    starving each other — a spinning fused-all-reduce grid of one rank cannot hold the CUs a
    peer needs to reach its side of the exchange (profiles/r05/rehearsal/). A masked process sees
    only its slice as the device's CU count, so launch shapes (and torch's random streams) follow
    the slice. Returns the mask set."""
    if os.environ.get("ROUNDTABLE_REHEARSAL_CU_SPLIT", "0") != "1" or world <= 1:
        return None
    ndev = max(1, torch.cuda.device_count())
    per_card = -(-world // ndev)
    if per_card <= 1:
        return None
    slot = local // ndev                       # ranks share cards round-robin (gpu = local % ndev)
    per = _card_cus() // per_card
    mask = hex(((1 << per) - 1) << (per * slot))
    os.environ["ROC_GLOBAL_CU_MASK"] = mask
    return mask


def init_cluster(prefer_gpu: bool = True, timeout_s: int = 1800) -> Cluster:
    """Initialize from torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); single process otherwise.
    ``timeout_s``: every collective of the world / control groups (and of the TP groups the SPMD
    commands create, knights/spmd.py) fails after it — the commands size it from the turn timeout
    (parallel/launch.py collective_timeout_s), so a stalled rank surfaces within minutes."""
    global _CLUSTER
    if _CLUSTER is not None:
        return _CLUSTER
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # Rehearsal mode (ROUNDTABLE_DIST_BACKEND=gloo): more ranks than GPUs share devices round-robin
    # and the data plane runs over gloo (RCCL refuses two ranks on one GPU) — lets a 1-GPU box run
    # the multi-rank GPU path (engines, hipGraphs, C1 exchange, TP collectives) end to end.
    forced = os.environ.get("ROUNDTABLE_DIST_BACKEND", "").strip().lower()
    if forced == "gloo" and prefer_gpu:
        rehearsal_cu_split(world, local)
    use_gpu = prefer_gpu and torch.cuda.is_available()
    gpu_index = local % max(1, torch.cuda.device_count()) if use_gpu and forced == "gloo" else local
    device = f"cuda:{gpu_index}" if use_gpu else "cpu"
    if use_gpu:
        torch.cuda.set_device(gpu_index)
    c = Cluster(rank=rank, world=world, local_rank=local, device=device, timeout_s=int(timeout_s))
    # a 1-rank world normally runs without a process group; ROUNDTABLE_DIST_BACKEND=nccl forces an
    # RCCL one (exercises the RCCL data plane on a 1-GPU box, tools/nccl_check.py)
    if world > 1 or (forced == "nccl" and use_gpu):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        backend = forced if forced in ("nccl", "gloo") else ("nccl" if use_gpu else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device(device)
        dist.init_process_group(**kw)
        c.backend = backend
        td = datetime.timedelta(seconds=timeout_s)
        c.cpu_group = dist.new_group(backend="gloo", timeout=td) if backend == "nccl" else dist.group.WORLD
        c.wait_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=WAIT_TIMEOUT_S))
        c.load_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=LOAD_TIMEOUT_S))
    _CLUSTER = c
    return c


def shutdown_cluster() -> None:
    global _CLUSTER
    if _CLUSTER is not None and dist.is_initialized():
        dist.destroy_process_group()
    _CLUSTER = None
