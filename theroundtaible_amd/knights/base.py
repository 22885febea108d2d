"""Knight backend seam.

The reference's only inference seam is ``BaseAdapter.execute(prompt, timeoutMs) ->
Promise<string>`` (`src/adapters/base.ts:10-29`). Here a backend additionally

* keys work by a per-knight *sequence* (``seq_key``) so an engine can keep each
  knight's KV cache resident across turns and rounds;
* exposes ``execute_many`` so knights hosted by the same engine are decoded as one
  batch (one hipGraph replay per token for all of them);
* returns :class:`TurnResult` with the generated token ids (the C1 token-id path)
  and per-turn metrics (prefill/decode tokens and ms).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

from ..consensus import parse_consensus
from ..prompt import PromptLike
from ..types import ConsensusBlock


@dataclass
class TurnRequest:
    seq_key: str
    prompt: PromptLike
    round: int = 0
    max_new_tokens: Optional[int] = None
    # optional: seq_key -> TurnResult of the turns already finished HERE  ->  the table's next
    # prompt as far as those results determine it (or None). A distributed pool calls it while
    # the C1 exchange of the remote results is in flight and prefetches that prefix.
    speculate: Optional[Callable[[Dict[str, "TurnResult"]], Optional[PromptLike]]] = None


@dataclass
class TurnResult:
    text: str
    ids: Optional[List[int]] = None
    tokenizer: Optional[str] = None
    metrics: Dict[str, Any] = field(default_factory=dict)
    # the same ids as a tensor on the engine's device (C1 all-gathers it without host staging)
    dev_ids: Optional[Any] = None


class KnightBackend:
    """Abstract backend; subclasses implement :meth:`_run`."""

    name: str = "knight"
    adapter_id: str = ""

    def is_available(self) -> bool:
        return True

    def max_source_chars(self) -> Optional[int]:
        """Source-context budget in chars; None = default 200K (base.ts:17-24)."""
        return None

    def parse_consensus(self, response: str, rnd: int) -> Optional[ConsensusBlock]:
        # NOTE: the block's knight defaults to the *backend* name, not the knight (base.ts:26-27).
        return parse_consensus(response, self.name, rnd)

    def execute(self, prompt: PromptLike, timeout_s: float, seq_key: str = "", rnd: int = 0) -> TurnResult:
        res = self.execute_many([TurnRequest(seq_key, prompt, rnd)], timeout_s)[0]
        if isinstance(res, BaseException):
            raise res
        return res

    def execute_many(self, reqs: Sequence[TurnRequest],
                     timeout_s: float) -> List[Union[TurnResult, BaseException]]:
        out: List[Union[TurnResult, BaseException]] = []
        for r in reqs:
            try:
                out.append(self._run(r, timeout_s))
            except Exception as e:  # noqa: BLE001 - surfaced per knight
                out.append(e)
        return out

    def group_key(self):
        """Backends with equal group keys are executed together (one batched decode)."""
        return id(self)

    def execute_group(self, pairs: Sequence[Tuple["KnightBackend", TurnRequest]],
                      timeout_s: float) -> List[Union[TurnResult, BaseException]]:
        out: List[Union[TurnResult, BaseException]] = []
        for backend, req in pairs:
            out.extend(backend.execute_many([req], timeout_s))
        return out

    def prefetch(self, seq_key: str, prompt_prefix: PromptLike) -> None:
        """Optional: ingest a known prefix of the knight's next prompt ahead of time."""

    def release(self, seq_key: str) -> None:
        """Optional: drop the resident state of one knight sequence."""

    def close(self) -> None:
        pass

    def _run(self, req: TurnRequest, timeout_s: float) -> TurnResult:  # pragma: no cover
        raise NotImplementedError


class BackendLock:
    """Serializes calls into one backend instance from orchestrator worker threads."""

    def __init__(self):
        self._lock = threading.Lock()

    def __enter__(self):
        self._lock.acquire()
        return self

    def __exit__(self, *a):
        self._lock.release()
