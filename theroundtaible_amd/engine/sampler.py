"""Sampling parameters (K6 does the work: csrc/sampling.hip)."""
from __future__ import annotations

import hashlib
from typing import Optional
from dataclasses import dataclass


@dataclass
class SamplingParams:
    temperature: float = 0.7
    top_p: float = 0.95
    top_k: int = 0
    seed: int = 0
    max_new_tokens: int = 512
    ignore_eos: bool = False
    stop_on_consensus: bool = True
    # teacher-forced text appended after the sampled tokens (knights/script.py scripted consensus)
    forced_tail: Optional[str] = None

    def seq_seed(self, seq_key: str) -> int:
        """Deterministic per (engine seed, knight): sample i of a knight depends only on (seed, knight, position)."""
        h = hashlib.sha256(f"{self.seed}:{seq_key}".encode()).digest()
        return int.from_bytes(h[:8], "little") & ((1 << 63) - 1)
