"""Schema types for config, consensus, sessions and persistence.

Parity: reference `src/types.ts:1-148`. Field names are kept byte-identical because
they are serialized to `.roundtable/*.json` and parsed out of model output.
Config objects keep the *raw* dict as well, so unknown fields (including the
MI355X engine extensions in ``adapter_config``) round-trip untouched.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field, asdict
from typing import Any, Dict, List, Optional


class _Undefined:
    """JS ``undefined``: a status update carrying it *removes* the key (JSON.stringify drops it)."""

    _inst = None

    def __new__(cls):
        if cls._inst is None:
            cls._inst = super().__new__(cls)
        return cls._inst

    def __repr__(self) -> str:  # pragma: no cover
        return "UNDEFINED"


UNDEFINED = _Undefined()


def dumps_js(obj: Any) -> str:
    """``JSON.stringify(obj, null, 2)`` equivalent (unicode kept, ints without ``.0``)."""

    def norm(o):
        if isinstance(o, float) and o.is_integer() and abs(o) < 2 ** 53:
            return int(o)
        if isinstance(o, dict):
            return {k: norm(v) for k, v in o.items() if v is not UNDEFINED}
        if isinstance(o, (list, tuple)):
            return [norm(v) for v in o]
        return o

    return json.dumps(norm(obj), indent=2, ensure_ascii=False)


@dataclass
class KnightConfig:
    name: str
    adapter: str
    capabilities: List[str]
    priority: float
    fallback: Optional[str] = None

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "KnightConfig":
        return cls(name=d.get("name"), adapter=d.get("adapter"),
                   capabilities=list(d.get("capabilities") or []),
                   priority=d.get("priority"), fallback=d.get("fallback"))

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {"name": self.name, "adapter": self.adapter,
                             "capabilities": list(self.capabilities), "priority": self.priority}
        if self.fallback:
            d["fallback"] = self.fallback
        return d


@dataclass
class RulesConfig:
    max_rounds: int = 5
    consensus_threshold: float = 9
    timeout_per_turn_seconds: float = 120
    escalate_to_user_after: int = 3
    auto_execute: bool = False
    ignore: List[str] = field(default_factory=lambda: [".git", "node_modules", "dist", "build", ".next"])
    # MI355X extensions. Reference semantics are the defaults.
    round_mode: str = "sequential"        # "sequential" (reference) | "parallel"
    prompt_layout: str = "reference"      # "reference" (reference shape) | "append" | "shared" (KV-friendly)
    # "literal" (every occurrence, verbatim) | "reference" (JS String.replace: first occurrence,
    # $-patterns expanded; prompt.py)
    placeholder_semantics: str = "literal"

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RulesConfig":
        r = cls()
        for k in ("max_rounds", "consensus_threshold", "timeout_per_turn_seconds",
                  "escalate_to_user_after", "auto_execute", "round_mode", "prompt_layout",
                  "placeholder_semantics"):
            if k in d and d[k] is not None:
                setattr(r, k, d[k])
        if isinstance(d.get("ignore"), list):
            r.ignore = list(d["ignore"])
        return r


@dataclass
class RoundtableConfig:
    version: str
    project: str
    language: str
    knights: List[KnightConfig]
    rules: RulesConfig
    chronicle: str
    adapter_config: Dict[str, Dict[str, Any]]
    raw: Dict[str, Any] = field(default_factory=dict, repr=False)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RoundtableConfig":
        return cls(version=d.get("version"), project=d.get("project", ""),
                   language=d.get("language", "nl"),
                   knights=[KnightConfig.from_dict(k) for k in d.get("knights") or []],
                   rules=RulesConfig.from_dict(d.get("rules") or {}),
                   chronicle=d.get("chronicle") or ".roundtable/chronicle.md",
                   adapter_config=dict(d.get("adapter_config") or {}), raw=d)


@dataclass
class ConsensusBlock:
    knight: str
    round: int
    consensus_score: float
    agrees_with: List[Any] = field(default_factory=list)
    pending_issues: List[str] = field(default_factory=list)
    proposal: Any = None
    files_to_modify: List[str] = field(default_factory=list)
    file_requests: List[Any] = field(default_factory=list)
    verify_commands: List[Any] = field(default_factory=list)

    def to_dict(self) -> Dict[str, Any]:
        d = asdict(self)
        if d["proposal"] is None:
            d.pop("proposal")
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ConsensusBlock":
        return cls(**{k: d[k] for k in cls.__dataclass_fields__ if k in d})


@dataclass
class RoundEntry:
    knight: str
    round: int
    response: str
    consensus: Optional[ConsensusBlock]
    timestamp: str
    # engine metrics for this turn (not part of the reference record; kept out of discussion.md)
    metrics: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> Dict[str, Any]:
        return {"knight": self.knight, "round": self.round, "response": self.response,
                "consensus": self.consensus.to_dict() if self.consensus else None,
                "timestamp": self.timestamp, "metrics": self.metrics}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RoundEntry":
        c = d.get("consensus")
        return cls(knight=d["knight"], round=d["round"], response=d["response"],
                   consensus=ConsensusBlock.from_dict(c) if c else None,
                   timestamp=d.get("timestamp", ""), metrics=d.get("metrics") or {})


SESSION_PHASES = ("discussing", "consensus_reached", "escalated", "applying", "completed")


@dataclass
class SessionResult:
    session_path: str
    consensus: bool
    rounds: int
    decision: Optional[str]
    blocks: List[ConsensusBlock]
    all_rounds: List[RoundEntry]
    unanimous_rejection: bool = False
    resolved_files: str = ""
    resolved_commands: str = ""
    lead_knight: Optional[str] = None


@dataclass
class ContinueOptions:
    """State for a "send back" continuation (types.ts:101-107)."""
    session_path: str
    all_rounds: List[RoundEntry]
    start_round: int
    resolved_files: str = ""
    resolved_commands: str = ""


MANIFEST_STATUSES = ("implemented", "partial", "deprecated")
DECREE_TYPES = ("rejected_no_apply", "deferred", "override_scope")
