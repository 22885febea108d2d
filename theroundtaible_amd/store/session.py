"""Session store: ``.roundtable/sessions/<UTC date>-<HHMM>-<slug>/``.

Byte formats follow the reference (`src/utils/session.ts:9-212`):
``topic.md``, ``status.json`` (2-space JSON, read-merge-write), ``discussion.md``
(rewritten after every round), ``decisions.md``.

Additions: ``rounds.jsonl`` is appended after every turn so a
crashed discussion can be resumed from disk (``discuss --continue``), and
``metrics.jsonl`` carries per-turn engine timings. Both are invisible to tools that
only know the reference format.
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..types import UNDEFINED, RoundEntry, dumps_js
from ..utils.atomic import atomic_write_text, file_lock, read_text
from ..utils.clock import iso_now


def slugify(text: str) -> str:
    s = re.sub(r"[^a-z0-9]+", "-", text.lower())
    s = re.sub(r"^-|-$", "", s)
    return s[:50]


def sessions_dir(project_root: str) -> str:
    return os.path.join(project_root, ".roundtable", "sessions")


def _initial_status() -> Dict[str, Any]:
    return {"phase": "discussing", "current_knight": None, "round": 0,
            "consensus_reached": False, "started_at": iso_now(), "updated_at": iso_now()}


def create_session(project_root: str, topic: str) -> str:
    now = iso_now()
    name = f"{now[:10]}-{now[11:16].replace(':', '')}-{slugify(topic)}"
    path = os.path.join(sessions_dir(project_root), name)
    os.makedirs(path, exist_ok=True)
    atomic_write_text(os.path.join(path, "topic.md"), f"# Topic\n\n{topic}\n")
    atomic_write_text(os.path.join(path, "status.json"), dumps_js(_initial_status()))
    return path


def render_discussion(rounds: List[RoundEntry]) -> str:
    lines: List[str] = ["# Discussion\n"]
    for e in rounds:
        lines.append(f"## Round {e.round} — {e.knight}")
        lines.append(f"*{e.timestamp}*\n")
        lines.append(e.response)
        lines.append("")
        c = e.consensus
        if c is not None:
            lines.append("**Consensus:**")
            score = c.consensus_score
            score_s = str(int(score)) if isinstance(score, float) and score.is_integer() else str(score)
            lines.append(f"- Score: {score_s}/10")
            if c.agrees_with:
                lines.append(f"- Agrees with: {', '.join(str(a) for a in c.agrees_with)}")
            if c.pending_issues:
                lines.append(f"- Pending: {', '.join(c.pending_issues)}")
        lines.append("\n---\n")
    return "\n".join(lines)


def write_discussion(session_path: str, rounds: List[RoundEntry]) -> None:
    atomic_write_text(os.path.join(session_path, "discussion.md"), render_discussion(rounds))


def render_decisions(topic: str, decision: str, rounds: List[RoundEntry]) -> str:
    knights: List[str] = []
    for r in rounds:
        if r.knight not in knights:
            knights.append(r.knight)
    # NOTE: "Rounds" counts *entries* (session.ts:106) — kept for byte compatibility.
    lines = ["# Decision\n", f"**Topic:** {topic}", f"**Knights:** {', '.join(knights)}",
             f"**Rounds:** {len(rounds)}", f"**Date:** {iso_now()[:10]}", "", "---\n", decision, ""]
    return "\n".join(lines)


def write_decisions(session_path: str, topic: str, decision: str, rounds: List[RoundEntry]) -> None:
    atomic_write_text(os.path.join(session_path, "decisions.md"), render_decisions(topic, decision, rounds))


def update_status(session_path: str, **updates: Any) -> Dict[str, Any]:
    """Read-merge-write of status.json under a file lock. ``UNDEFINED`` values delete keys."""
    p = os.path.join(session_path, "status.json")
    with file_lock(p):
        current: Dict[str, Any]
        if os.path.exists(p):
            try:
                current = json.loads(read_text(p))
            except (OSError, ValueError):
                current = _initial_status()
        else:
            current = _initial_status()
        merged = dict(current)
        for k, v in updates.items():
            if v is UNDEFINED:
                merged.pop(k, None)
            else:
                merged[k] = v
        merged["updated_at"] = iso_now()
        atomic_write_text(p, dumps_js(merged))
    return merged


def read_status(session_path: str) -> Optional[Dict[str, Any]]:
    p = os.path.join(session_path, "status.json")
    if not os.path.exists(p):
        return None
    try:
        return json.loads(read_text(p))
    except (OSError, ValueError):
        return None


@dataclass
class SessionInfo:
    name: str
    path: str
    status: Optional[Dict[str, Any]]
    topic: Optional[str]


def list_sessions(project_root: str) -> List[SessionInfo]:
    d = sessions_dir(project_root)
    if not os.path.isdir(d):
        return []
    out: List[SessionInfo] = []
    for name in os.listdir(d):
        path = os.path.join(d, name)
        if not os.path.isdir(path):
            continue
        topic = None
        tp = os.path.join(path, "topic.md")
        if os.path.exists(tp):
            raw = read_text(tp)
            m = re.search(r"^# Topic\s*\n\n(.+)", raw, re.M)
            topic = (m.group(1).strip() if m else "") or raw.strip()
        out.append(SessionInfo(name, path, read_status(path), topic))
    out.sort(key=lambda s: s.name, reverse=True)
    return out


def find_latest_session(project_root: str) -> Optional[SessionInfo]:
    s = list_sessions(project_root)
    return s[0] if s else None


# ---- resume / metrics (new) -------------------------------------------------------------

def append_round_entry(session_path: str, entry: RoundEntry) -> None:
    p = os.path.join(session_path, "rounds.jsonl")
    with file_lock(p), open(p, "a", encoding="utf-8") as f:
        f.write(json.dumps(entry.to_dict(), ensure_ascii=False) + "\n")
        f.flush()
        os.fsync(f.fileno())


def load_round_entries(session_path: str) -> List[RoundEntry]:
    p = os.path.join(session_path, "rounds.jsonl")
    if not os.path.exists(p):
        return []
    out: List[RoundEntry] = []
    for line in read_text(p).splitlines():
        line = line.strip()
        if not line:
            continue
        try:
            out.append(RoundEntry.from_dict(json.loads(line)))
        except (ValueError, KeyError):
            break  # torn tail from a crash: keep the prefix
    return out


def append_metrics(session_path: str, record: Dict[str, Any]) -> None:
    p = os.path.join(session_path, "metrics.jsonl")
    with open(p, "a", encoding="utf-8") as f:
        f.write(json.dumps(record, ensure_ascii=False) + "\n")
