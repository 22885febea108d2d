"""Engine-backed knights: every reference adapter id resolves to a locally hosted model.

``claude-cli`` / ``gemini-cli`` / ``openai-cli`` / ``*-api`` / ``local-llm*`` all map
to an :class:`EngineBackend` (`src/utils/adapters.ts:15-56` is the reference
factory). Backends whose effective engine settings (model, weights, dtype, device)
are equal share ONE :class:`~theroundtaible_amd.engine.engine.Engine`, and the
orchestrator batches their knights into one decode (``group_key``).
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence, Tuple, Union

from ..engine.engine import Engine, EngineConfig, Turn
from ..engine.sampler import SamplingParams
from .base import KnightBackend, TurnRequest, TurnResult
from .script import ConsensusScript

ADAPTER_DISPLAY_NAMES = {
    "claude-cli": "Claude", "claude-api": "Claude", "gemini-cli": "Gemini", "gemini-api": "Gemini",
    "openai-cli": "GPT", "openai-api": "GPT",
}


class EngineBackend(KnightBackend):
    def __init__(self, name: str, adapter_id: str, engine: Engine, params: SamplingParams,
                 lock: Optional[threading.Lock] = None, script: Optional[ConsensusScript] = None):
        self.name = name
        self.adapter_id = adapter_id
        self.engine = engine
        self.params = params
        self.lock = lock or threading.Lock()
        self.script = script

    def group_key(self):
        return id(self.engine)

    def is_available(self) -> bool:
        return self.engine.healthy

    def max_source_chars(self) -> Optional[int]:
        return self.engine.max_source_chars()

    def _turn(self, req: TurnRequest, timeout_s: float) -> Turn:
        p = self.params
        if req.max_new_tokens:
            p = SamplingParams(**{**p.__dict__, "max_new_tokens": int(req.max_new_tokens)})
        if self.script is not None:   # scripted consensus: free tokens, then the forced tail
            knight = req.seq_key.rsplit("/", 1)[-1].split(":", 1)[-1]
            p = SamplingParams(**{**p.__dict__, "max_new_tokens": min(p.max_new_tokens, self.script.free_tokens),
                                  "stop_on_consensus": False,
                                  "forced_tail": self.script.tail(knight, req.round, req.seq_key)})
        return Turn(req.seq_key, req.prompt, p, timeout_s)

    def execute_group(self, pairs: Sequence[Tuple["EngineBackend", TurnRequest]],
                      timeout_s: float) -> List[Union[TurnResult, BaseException]]:
        """Run requests of several backends that share this engine as one batch."""
        turns = [b._turn(r, timeout_s) for b, r in pairs]
        with self.lock:
            outs = self.engine.run_turns(turns)
        res: List[Union[TurnResult, BaseException]] = []
        for o in outs:
            if o.error is not None:
                res.append(o.error)
            else:
                res.append(TurnResult(o.text, o.ids, self.engine.tokenizer.family, dict(o.metrics), o.dev_ids))
        return res

    def execute_many(self, reqs: Sequence[TurnRequest], timeout_s: float):
        return self.execute_group([(self, r) for r in reqs], timeout_s)

    def prefetch(self, seq_key: str, prompt_prefix) -> None:
        """Prefill the shared (table) part of a predicted next prompt now (Engine.warm_shared)."""
        with self.lock:
            self.engine.warm_shared(prompt_prefix)

    def release(self, seq_key: str) -> None:
        with self.lock:
            self.engine.release(seq_key)


class EnginePool:
    """Process-local engines keyed by effective settings (one per model x device)."""

    def __init__(self):
        self.engines: Dict[tuple, Engine] = {}
        self.locks: Dict[tuple, threading.Lock] = {}

    def get(self, ecfg: EngineConfig, defer_kv: bool = False) -> Tuple[Engine, threading.Lock]:
        """``defer_kv``: load weights only; :meth:`finalize` sizes the KV pools afterwards."""
        key = (ecfg.model, ecfg.weights, ecfg.dtype, ecfg.device, ecfg.block_size)
        if key not in self.engines:
            if defer_kv and ecfg.num_blocks is None and ecfg.kv_budget_bytes is None:
                ecfg.defer_kv = True
            self.engines[key] = Engine(ecfg)
            self.locks[key] = threading.Lock()
        return self.engines[key], self.locks[key]

    def finalize(self) -> Dict[str, List[int]]:
        """Split each GPU's free HBM between the engines placed on it (once every engine's weights
        are resident), instead of the first engine taking ``kv_cache_fraction`` of everything:
        equal bytes per engine. Returns {device: [kv tokens per engine]}."""
        import torch
        by_dev: Dict[str, List[Engine]] = {}
        for e in self.engines.values():
            if not e.kv_allocated:
                by_dev.setdefault(str(e.device), []).append(e)
        out: Dict[str, List[int]] = {}
        for dev, engines in by_dev.items():
            if engines[0].on_gpu:
                free, _ = torch.cuda.mem_get_info(engines[0].device)
                frac = engines[0].ecfg.kv_cache_fraction
                share = max(0, int(free * frac) - (2 << 30) * len(engines)) // len(engines)
                for e in engines:
                    e.allocate_kv(share)
            else:
                for e in engines:
                    e.allocate_kv()
            out[dev] = [e.kv_capacity_tokens for e in engines]
        return out

    def close(self) -> None:
        self.engines.clear()
