"""C1: exchange every knight's turn output between ranks after a (parallel) round.

Token ids travel as one padded ``int32`` tensor per rank through
``all_gather_into_tensor`` on the default process group — RCCL over xGMI on GPUs
(gloo in CPU CI). Each rank contributes only the knights it *leads* (the first rank
of a knight's TP group); ~2 KB per knight, so the collective is latency-bound and
one call per round suffices. Metadata (errors, metrics, text for backends without
token ids) rides the gloo control group.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .cluster import Cluster

# (slot, ids) pairs contributed by this rank
Contribution = List[Tuple[int, List[int]]]


class TokenExchange:
    """C1 with static shapes: every rank contributes a ``[rows, width]`` int32 buffer (rows = the
    most knights any rank leads, from the placement; width = the reply-length cap + 2), so no
    shape agreement round is needed. The all-gather is issued asynchronously (RCCL on GPUs, on
    its own stream) and the caller overlaps it with the gloo metadata exchange and with the
    speculative prefill of the next prompt (knights/distributed.py); :meth:`wait` returns
    ``{slot: ids}``. Replies longer than the cap take :func:`exchange_token_ids`.

    Device-resident path: when every contribution carries its ids as a device
    tensor (``TurnResult.dev_ids``: a slice of the decode graph's token buffer), the send buffer is
    assembled ON the device (fills + device-to-device copies, no host round trip) and the
    all-gather reads it straight away; only the gathered result is copied back, into pinned
    memory, after the overlapped work. Host-only contributions go through a pinned staging
    buffer and an asynchronous copy."""

    def __init__(self, cluster: Cluster, rows: int, width: int, device: str):
        self.cluster, self.rows, self.width = cluster, max(1, rows), width + 2
        self.dev = device if cluster.backend == "nccl" else "cpu"
        self._src = torch.full((self.rows, self.width), -1, dtype=torch.int32, device=self.dev)
        self._out = torch.empty((cluster.world * self.rows, self.width), dtype=torch.int32, device=self.dev)
        on_dev = torch.device(self.dev).type == "cuda"
        self._stage = torch.empty((self.rows, self.width), dtype=torch.int32, pin_memory=on_dev)
        self._host = torch.empty((cluster.world * self.rows, self.width), dtype=torch.int32, pin_memory=on_dev)
        self._work = None
        self.device_path = 0    # contributions assembled on the device (observability / tests)

    def fits(self, mine: Contribution) -> bool:
        return len(mine) <= self.rows and all(len(c[1]) + 2 <= self.width for c in mine)

    def start(self, mine) -> None:
        """``mine``: (slot, ids) or (slot, ids, dev_ids) per knight this rank leads."""
        devs = [c[2] if len(c) > 2 else None for c in mine]
        if mine and all(d is not None for d in devs):
            src = self._src
            src.fill_(-1)
            cur = torch.cuda.current_stream(src.device) if src.is_cuda else None
            for r, ((slot, ids, *_), d) in enumerate(zip(mine, devs)):
                src[r, 0] = slot
                src[r, 1] = len(ids)
                if len(ids):
                    if cur is not None and d.is_cuda:
                        # the ids were written on the engine's stream: order this copy after them
                        # and keep their memory alive until this stream has read it
                        ev = getattr(d, "ready_event", None)
                        if ev is not None:
                            cur.wait_event(ev)
                        d.record_stream(cur)
                    src[r, 2:2 + len(ids)].copy_(d.reshape(-1)[:len(ids)].to(src.device, non_blocking=True))
            self.device_path += 1
        else:
            buf = self._stage
            buf.fill_(-1)
            for r, (slot, ids, *_) in enumerate(mine):
                buf[r, 0] = slot
                buf[r, 1] = len(ids)
                if ids:
                    buf[r, 2:2 + len(ids)] = torch.as_tensor(ids, dtype=torch.int32)
            self._src.copy_(buf, non_blocking=True)   # pinned: truly asynchronous
        self._work = dist.all_gather_into_tensor(self._out, self._src, async_op=True)

    def wait(self) -> Dict[int, List[int]]:
        self._work.wait()
        self._work = None
        if self._out.is_cuda:
            self._host.copy_(self._out, non_blocking=True)
            torch.cuda.current_stream(self._out.device).synchronize()
            host = self._host
        else:
            host = self._out
        res: Dict[int, List[int]] = {}
        for row in host.tolist():
            slot, n = row[0], row[1]
            if slot >= 0:
                res[slot] = row[2:2 + n]
        return res


def exchange_token_ids(cluster: Cluster, mine: Contribution, device: str) -> Dict[int, List[int]]:
    """All-gather ragged token-id lists keyed by request slot. Returns {slot: ids} for all ranks."""
    if not cluster.distributed:
        return {s: list(ids) for s, ids in mine}
    # agree on the padded shape (tiny gloo all-reduce of (rows, max_len))
    shape = torch.tensor([len(mine), max((len(i) for _, i in mine), default=0)], dtype=torch.int64)
    dist.all_reduce(shape, op=dist.ReduceOp.MAX, group=cluster.cpu_group)
    rows, width = int(shape[0]), int(shape[1]) + 2
    if rows == 0:
        return {}
    buf = torch.full((rows, width), -1, dtype=torch.int32)
    for r, (slot, ids) in enumerate(mine):
        buf[r, 0] = slot
        buf[r, 1] = len(ids)
        if ids:
            buf[r, 2:2 + len(ids)] = torch.tensor(ids, dtype=torch.int32)
    use_dev = device if cluster.backend == "nccl" else "cpu"
    src = buf.to(use_dev)
    out = torch.empty((cluster.world * rows, width), dtype=torch.int32, device=use_dev)
    dist.all_gather_into_tensor(out, src)
    host = out.cpu()
    res: Dict[int, List[int]] = {}
    for row in host.tolist():
        slot, n = row[0], row[1]
        if slot >= 0:
            res[slot] = row[2:2 + n]
    return res
