"""King's decree log (`src/utils/decree-log.ts:15-103`).

Unlike the snapshot (where ``addDecreeEntry`` is imported but never called,
`src/commands/discuss.ts:7`), decrees are *written* here: ``rejected_no_apply`` /
``deferred`` from the King's decree prompt after a discussion and ``override_scope``
from ``apply --override-scope`` (TODO.md:95-100).
"""
from __future__ import annotations

import json
import os
import re
from typing import Any, Dict, List, Optional

from ..utils.atomic import atomic_write_text, file_lock, read_text
from ..utils.clock import iso_now
from ..types import dumps_js

DECREE_LOG_PATH = os.path.join(".roundtable", "decree-log.json")


def empty_log() -> Dict[str, Any]:
    return {"version": "1.0", "entries": []}


def read_decree_log(project_root: str) -> Dict[str, Any]:
    p = os.path.join(project_root, DECREE_LOG_PATH)
    if not os.path.exists(p):
        return empty_log()
    try:
        d = json.loads(read_text(p))
        if isinstance(d, dict) and d.get("version") == "1.0" and isinstance(d.get("entries"), list):
            return d
    except (OSError, ValueError):
        pass
    return empty_log()


def next_decree_id(log: Dict[str, Any]) -> str:
    best = 0
    for e in log["entries"]:
        m = re.match(r"^decree-(\d+)$", str(e.get("id", "")))
        if m:
            best = max(best, int(m.group(1)))
    return f"decree-{best + 1:03d}"


def add_decree_entry(project_root: str, type_: str, session: str, topic: str,
                     reason: Optional[str] = None) -> Dict[str, Any]:
    p = os.path.join(project_root, DECREE_LOG_PATH)
    with file_lock(p):
        log = read_decree_log(project_root)
        entry = {"id": next_decree_id(log), "type": type_, "session": session, "topic": topic,
                 "reason": (reason or "").strip() or "No reason provided", "revoked": False,
                 "date": iso_now()}
        log["entries"].append(entry)
        atomic_write_text(p, dumps_js(log) + "\n")
    return entry


def active_decrees(log: Dict[str, Any], max_n: int = 5) -> List[Dict[str, Any]]:
    return [e for e in log["entries"] if not e.get("revoked")][-max_n:]


def format_decrees_for_prompt(decrees: List[Dict[str, Any]]) -> str:
    if not decrees:
        return ""
    lines = ["KING'S DECREES (afgewezen beslissingen — stel NIET opnieuw voor tenzij je de afwijsreden expliciet adresseert):"]
    for d in decrees:
        topic = d["topic"] if len(d["topic"]) <= 50 else d["topic"][:47] + "..."
        lines.append(f'- [{d["id"]}] {d["type"].upper()} — "{topic}": "{d["reason"]}" ({d["date"][:10]})')
    return "\n".join(lines)
