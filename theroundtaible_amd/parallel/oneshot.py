"""K9: one-shot all-reduce for tensor-parallel decode (csrc/oneshot_ar.hip).

Decode all-reduces are latency-bound (``[B, hidden]`` bf16, 16 KB at B = 1 on Llama-3-70B, two
per layer). On an MI355X node every GPU has a dedicated xGMI link to each peer, so instead of
RCCL's ring (world-1 dependent steps) each rank pushes its partial into every peer's IPC-mapped
receive buffer in one step and sums the copies locally. Larger messages (prefill) stay on RCCL.

Set-up is collective over the TP group: each rank allocates uncached receive/flag buffers,
the 128-byte IPC handles are exchanged with ``all_gather_object``, and every rank maps its
peers'. The launch itself is hipGraph-capturable (device-side call counter).
``ROUNDTABLE_ONESHOT_AR=0`` disables it (RCCL everywhere).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

DEFAULT_CAP_ELEMS = 16 * 8192     # M <= 16 decode rows x hidden 8192 (Llama-3-70B)


def enabled_by_env() -> bool:
    return os.environ.get("ROUNDTABLE_ONESHOT_AR", "1") != "0"


class OneShotAllReduce:
    """Use :func:`try_create` (collective); the constructor wraps an already-opened comm."""

    def __init__(self, nat, comm_id: int, rank: int, world: int, cap_elems: int):
        self._nat, self.id = nat, comm_id
        self.world, self.rank, self.cap = world, rank, cap_elems

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
    return OneShotAllReduce(nat, comm_id, rank, world, cap_elems)
