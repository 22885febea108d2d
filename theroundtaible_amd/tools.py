"""Knight ``file_requests`` tool (`src/orchestrator.ts:164-222`).

Workspace-relative paths only (no traversal, no absolute paths, ignore patterns
denied), optional ``path:a-b`` line ranges, otherwise the first 200 lines.
"""
from __future__ import annotations

import os
import posixpath
import re
from typing import Iterable, List

_RANGE = re.compile(r"^(.+?):(\d+)-(\d+)$")


def _normalize(p: str) -> str:
    # node's path.normalize: collapse '.', resolvable '..', duplicate slashes; keep leading '..'.
    if not p:
        return "."
    n = posixpath.normpath(p.replace("\\", "/"))
    if p.endswith("/") and not n.endswith("/"):
        n += "/"
    return n


def resolve_file_requests(requests: Iterable[str], root: str, ignore: List[str]) -> str:
    results: List[str] = []
    for req in list(requests)[:4]:
        req = str(req)
        m = _RANGE.match(req)
        path = m.group(1) if m else req
        start = int(m.group(2)) if m else None
        end = int(m.group(3)) if m else None
        norm = _normalize(path).replace("\\", "/")
        if ".." in norm or norm.startswith("/"):
            results.append(f"[DENIED] {req} — path traversal not allowed")
            continue
        if any(norm.startswith(p) or f"/{p}/" in norm for p in ignore):
            results.append(f"[DENIED] {req} — matches ignore pattern")
            continue
        full = os.path.join(root, norm)
        if not os.path.exists(full):
            results.append(f"[NOT FOUND] {req}")
            continue
        try:
            with open(full, "r", encoding="utf-8", errors="replace", newline="") as f:
                lines = f.read().split("\n")
        except OSError:
            results.append(f"[ERROR] {req} — could not read file")
            continue
        if start is not None and end is not None:
            excerpt = "\n".join(lines[max(0, start - 1):min(len(lines), end)])
        else:
            excerpt = "\n".join(lines[:200])
            if len(lines) > 200:
                excerpt += f"\n...({len(lines) - 200} more lines)"
        results.append(f"### {req}\n```\n{excerpt}\n```")
    return "\n\n".join(results)
