"""Paged KV cache + block manager (the resident per-knight memory).

Layout per layer (see ``ops/reference.py``): ``K [num_blocks, Hkv, BS, D]`` and
``V [num_blocks, Hkv, D, BS]`` — both one allocation ``[L, num_blocks, Hkv, BS*D]``.
Blocks are handed out from a free list with reference counts, so a sequence can be
forked (copy-on-write share of a prefix: ``fork``) and truncated back to any token
count (``truncate``), which is how a knight's cache is rolled back to the longest
common prefix with its next prompt.

Sizing for 288 GB HBM: the cache takes ``kv_cache_fraction`` of what is free after
weights, e.g. ~230 GB on an 8B knight's GPU = 1.8M tokens at 128 KiB/token — every
knight's whole discussion stays resident across rounds with room to spare.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch


class KVCacheOOM(RuntimeError):
    """Raised when the block pool is exhausted (classified as ``oom`` by the orchestrator)."""


class BlockAllocator:
    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self.free: List[int] = list(range(num_blocks - 1, -1, -1))
        self.ref = [0] * num_blocks

    def alloc(self) -> int:
        if not self.free:
            raise KVCacheOOM("KV cache out of memory: no free blocks")
        b = self.free.pop()
        self.ref[b] = 1
        return b

    def incref(self, b: int) -> None:
        self.ref[b] += 1

    def release(self, b: int) -> None:
        self.ref[b] -= 1
        if self.ref[b] == 0:
            self.free.append(b)
        elif self.ref[b] < 0:  # pragma: no cover - logic error guard
            raise RuntimeError(f"double free of KV block {b}")

    @property
    def num_free(self) -> int:
        return len(self.free)


@dataclass
class SeqState:
    """One knight's resident sequence: the token ids whose K/V are in ``blocks``."""
    key: str
    tokens: List[int] = field(default_factory=list)
    blocks: List[int] = field(default_factory=list)

    @property
    def length(self) -> int:
        return len(self.tokens)


class PagedKVCache:
    def __init__(self, n_layers: int, n_kv_heads: int, head_dim: int, num_blocks: int, block_size: int,
                 device, dtype=torch.bfloat16):
        self.n_layers, self.n_kv_heads, self.head_dim = n_layers, n_kv_heads, head_dim
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.device = device
        self.dtype = dtype
        shape = (n_layers, num_blocks, n_kv_heads, block_size * head_dim)
        # zero-init: masked tail keys of a partial block must be finite (0 * NaN = NaN in P.V)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)
        self.alloc = BlockAllocator(num_blocks)
        self.seqs: Dict[str, SeqState] = {}

    # views in the kernel layouts
    def k_layer(self, l: int) -> torch.Tensor:
        return self.k[l].view(self.num_blocks, self.n_kv_heads, self.block_size, self.head_dim)

    def v_layer(self, l: int) -> torch.Tensor:
        return self.v[l].view(self.num_blocks, self.n_kv_heads, self.head_dim, self.block_size)

    @staticmethod
    def bytes_per_block(n_layers, n_kv_heads, head_dim, block_size, dtype_bytes=2) -> int:
        return 2 * n_layers * n_kv_heads * head_dim * block_size * dtype_bytes

    # ---- sequence management ------------------------------------------------------------
    def seq(self, key: str) -> SeqState:
        s = self.seqs.get(key)
        if s is None:
            s = self.seqs[key] = SeqState(key)
        return s

    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    # positions a sequence may reach (the model's RoPE table / position embeddings and the block
    # tables are sized by it); None = unbounded. Past it a kernel would index beyond those tables,
    # so the turn fails here, on the host, like any other KV exhaustion (kind "oom").
    max_tokens: Optional[int] = None

    def ensure_capacity(self, s: SeqState, n_tokens: int) -> None:
        """Grow ``s.blocks`` to hold ``n_tokens`` (copy-on-write if the tail block is shared)."""
        if self.max_tokens is not None and n_tokens > self.max_tokens:
            raise KVCacheOOM(f"context of {n_tokens} tokens exceeds the model's {self.max_tokens} positions")
        need = self.blocks_needed(n_tokens)
        if s.blocks and self.alloc.ref[s.blocks[-1]] > 1 and s.length % self.block_size:
            self._cow_tail(s)
        while len(s.blocks) < need:
            s.blocks.append(self.alloc.alloc())

    def _cow_tail(self, s: SeqState) -> None:
        old = s.blocks[-1]
        new = self.alloc.alloc()
        self.copy_blocks([old], [new])
        self.alloc.release(old)
        s.blocks[-1] = new

    def copy_blocks(self, src: List[int], dst: List[int]) -> None:
        """K8 (csrc/kv_copy.hip): whole-block copies across every layer of K and V, one launch."""
        from .. import ops
        ops.kv_block_copy(self.k.view(self.n_layers, self.num_blocks, -1),
                          self.v.view(self.n_layers, self.num_blocks, -1), src, dst)

    def truncate(self, s: SeqState, n_tokens: int) -> None:
        n_tokens = max(0, min(n_tokens, s.length))
        keep = self.blocks_needed(n_tokens)
        for b in s.blocks[keep:]:
            self.alloc.release(b)
        del s.blocks[keep:]
        del s.tokens[n_tokens:]

    def free_seq(self, key: str) -> None:
        s = self.seqs.pop(key, None)
        if s is not None:
            for b in s.blocks:
                self.alloc.release(b)

    def fork(self, src: str, dst: str, copy: bool = False) -> SeqState:
        """``dst`` starts as ``src``. Default: share the blocks (refcounted prefix sharing; a writer
        copies-on-write its tail). ``copy=True``: a deep snapshot in fresh blocks (K8 batch copy),
        e.g. a continuation branch that must survive the live sequence being rolled back."""
        self.free_seq(dst)
        a = self.seqs[src]
        if copy:
            new = [self.alloc.alloc() for _ in a.blocks]
            self.copy_blocks(list(a.blocks), new)
            b = self.seqs[dst] = SeqState(dst, list(a.tokens), new)
            return b
        b = self.seqs[dst] = SeqState(dst, list(a.tokens), list(a.blocks))
        for blk in b.blocks:
            self.alloc.incref(blk)
        return b

    def slots(self, s: SeqState, start: int, end: int) -> List[int]:
        bs = self.block_size
        return [s.blocks[p // bs] * bs + (p % bs) for p in range(start, end)]
