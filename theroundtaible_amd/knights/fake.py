"""Deterministic scripted backend + fault injection (the reference has no mock adapter).

``script`` maps ``(seq_key, round)`` -> response, ``seq_key`` -> list of responses
(consumed in order), or is a callable ``(seq_key, prompt_text, call_index) -> str``.
Fault injection: ``faults`` maps call index (0-based, per seq_key) -> ``"raise:<msg>"``,
``"hang"`` (sleeps past the timeout and raises a timeout) or ``"oom"``.
"""
from __future__ import annotations

import json
import time
from collections import defaultdict
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

from ..errors import AdapterError, EngineTimeout
from ..prompt import PromptLike, prompt_text
from .base import KnightBackend, TurnRequest, TurnResult

Script = Union[Dict[Any, Any], Callable[[str, str, int], str]]


def consensus_reply(score: float, text: str = "Mijn standpunt.", **extra: Any) -> str:
    block = {"consensus_score": score, "agrees_with": extra.pop("agrees_with", []),
             "pending_issues": extra.pop("pending_issues", [])}
    block.update(extra)
    return f"{text}\n\n```json\n{json.dumps(block, indent=2)}\n```"


class FakeBackend(KnightBackend):
    def __init__(self, name: str = "Fake", script: Optional[Script] = None,
                 faults: Optional[Dict[Tuple[str, int], str]] = None, available: bool = True,
                 latency_s: float = 0.0, max_chars: Optional[int] = None, adapter_id: str = "fake"):
        self.name = name
        self.adapter_id = adapter_id
        self.script = script if script is not None else {}
        self.faults = faults or {}
        self.available = available
        self.latency_s = latency_s
        self.max_chars = max_chars
        self.calls: Dict[str, int] = defaultdict(int)
        self.prompts: List[Tuple[str, str]] = []
        self.prompt_objs: List[Tuple[str, object]] = []   # the Prompt objects (segments, shared split)

    def is_available(self) -> bool:
        return self.available

    def max_source_chars(self) -> Optional[int]:
        return self.max_chars

    def _run(self, req: TurnRequest, timeout_s: float) -> TurnResult:
        seq_key, prompt = req.seq_key.split("/")[-1], req.prompt   # drop a table prefix "t3/"
        idx = self.calls[seq_key]
        self.calls[seq_key] += 1
        text = prompt_text(prompt)
        self.prompts.append((seq_key, text))
        self.prompt_objs.append((seq_key, prompt))
        fault = self.faults.get((seq_key, idx))
        if fault == "hang":
            time.sleep(min(timeout_s, 0.05))
            raise EngineTimeout(self.name, f"turn timed out after {timeout_s}s")
        if fault == "oom":
            raise AdapterError(self.name, "HIP out of memory while growing KV", kind="oom")
        if fault and fault.startswith("raise:"):
            raise RuntimeError(fault[6:])
        if self.latency_s:
            time.sleep(self.latency_s)
        s = self.script
        if callable(s):
            out = s(seq_key, text, idx)
        elif isinstance(s, dict):
            rnd = req.round
            if (seq_key, rnd) in s:
                out = s[(seq_key, rnd)]
            elif seq_key in s:
                v = s[seq_key]
                out = v[min(idx, len(v) - 1)] if isinstance(v, list) else v
            else:
                out = consensus_reply(5)
        else:
            out = str(s)
        return TurnResult(text=out, metrics={"backend": "fake", "prompt_chars": len(text)})

