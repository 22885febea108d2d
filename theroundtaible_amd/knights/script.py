"""Scripted consensus: a deterministic forced tail for engine knights (SURVEY §7.3 hard part 3).

Random-init weights never write a parseable consensus block, so on their own they can never
exercise the consensus paths the reference is built around (`src/consensus.ts:118-145`
parse, `:217-239` consensus / negative consensus, the early exit after a full round,
`roundtable apply`). With ``engine.scripted_consensus`` set, every engine knight samples
``free_tokens`` tokens freely and then the engine *teacher-forces* a tail (prefilled into the
knight's KV like any generated text, so the transcript and the caches stay consistent):

* discussion turns: a fenced consensus JSON whose score follows ``scores`` by round
  (``[6, 9]`` = no agreement in round 1, consensus in round 2; ``reject: true`` = 2/10 from
  round ``reject_round`` on, i.e. unanimous rejection), ``files_to_modify`` = ``files``;
* ``apply`` turns (sequence key ``apply:``): an RTDIFF/1 block that CREATEs the first
  ``NEW:`` file of ``files`` with the decision summary — a valid, in-scope edit;
* ``code-red`` doctors (``codered:``): a doctor JSON with one agreed ``root_cause_key``.

Config (``.roundtable/config.json``)::

    "engine": {"scripted_consensus": {"free_tokens": 48, "scores": [6, 9],
                                      "files": ["NEW:docs/roundtable-besluit.md"]}}
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class ConsensusScript:
    free_tokens: int = 48
    scores: List[float] = field(default_factory=lambda: [6, 9])
    files: List[str] = field(default_factory=lambda: ["NEW:docs/roundtable-besluit.md"])
    reject: bool = False
    reject_round: int = 1

    @classmethod
    def from_config(cls, d: Optional[Dict[str, Any]]) -> Optional["ConsensusScript"]:
        if not d:
            return None
        if d is True:
            return cls()
        return cls(free_tokens=int(d.get("free_tokens", 48)), scores=list(d.get("scores", [6, 9])),
                   files=list(d.get("files", ["NEW:docs/roundtable-besluit.md"])),
                   reject=bool(d.get("reject", False)), reject_round=int(d.get("reject_round", 1)))

    def score(self, rnd: int) -> float:
        if self.reject and rnd >= self.reject_round:
            return 2
        if not self.scores:
            return 9
        return self.scores[min(max(rnd, 1), len(self.scores)) - 1]

    def tail(self, knight: str, rnd: int, seq_key: str = "") -> str:
        key = seq_key.rsplit("/", 1)[-1]
        if key.startswith("apply:"):
            return self.apply_tail(knight)
        if key.startswith("codered:"):
            return self.codered_tail(rnd)
        s = self.score(rnd)
        block = {"consensus_score": s, "agrees_with": ["gedeelde KV-cache per tafel"] if s >= 6 else [],
                 "pending_issues": [] if s >= 9 else ["meetbare winst per ronde aantonen"],
                 "proposal": f"{knight}: bewaar de gedeelde transcript-KV een keer per GPU en meet het.",
                 "files_to_modify": list(self.files) if s >= 9 else []}
        return "\n\n```json\n" + json.dumps(block, ensure_ascii=False) + "\n```\n"

    def apply_tail(self, knight: str) -> str:
        new = next((f[4:] for f in self.files if f.upper().startswith("NEW:")), None)
        if new is None:
            return "\nRTDIFF/1\n"
        body = (f"# Besluit van de ronde tafel\n\nLead knight: {knight}.\n"
                "Bewaar de gedeelde transcript-KV een keer per GPU.\n")
        return f"\nRTDIFF/1\nFILE: NEW:{new}\nCREATE\n<<<\n{body}>>>\n"

    def codered_tail(self, rnd: int) -> str:
        block = {"confidence_score": 9 if rnd >= 2 else 6, "root_cause_key": "kv-cache-exhausted",
                 "evidence": ["resident KV groeit elke ronde"], "rules_out": ["tokenizer"],
                 "confirms": ["kv_capacity_tokens"], "file_requests": [], "next_test": "meet kv_blocks_used"}
        return "\n\n```json\n" + json.dumps(block, ensure_ascii=False) + "\n```\n"
