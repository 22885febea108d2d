"""Implementation manifest (`src/utils/manifest.ts:13-183`): what the table has already built."""
from __future__ import annotations

import json
import os
import re
from typing import Any, Dict, List, Optional

from ..types import dumps_js
from ..utils.atomic import atomic_write_text, file_lock, read_text
from ..utils.clock import iso_now

MANIFEST_PATH = os.path.join(".roundtable", "manifest.json")


def empty_manifest() -> Dict[str, Any]:
    return {"version": "1.0", "last_updated": iso_now(), "features": []}


def read_manifest(project_root: str) -> Dict[str, Any]:
    p = os.path.join(project_root, MANIFEST_PATH)
    if not os.path.exists(p):
        return empty_manifest()
    try:
        m = json.loads(read_text(p))
        if not isinstance(m, dict) or not isinstance(m.get("features"), list):
            return empty_manifest()
        return m
    except (OSError, ValueError):
        return empty_manifest()


def write_manifest(project_root: str, manifest: Dict[str, Any]) -> None:
    manifest["last_updated"] = iso_now()
    atomic_write_text(os.path.join(project_root, MANIFEST_PATH), dumps_js(manifest))


def add_manifest_entry(project_root: str, entry: Dict[str, Any]) -> None:
    p = os.path.join(project_root, MANIFEST_PATH)
    with file_lock(p):
        m = read_manifest(project_root)
        for i, f in enumerate(m["features"]):
            if f.get("id") == entry["id"]:
                m["features"][i] = entry
                break
        else:
            m["features"].append(entry)
        write_manifest(project_root, m)


def deprecate_feature(project_root: str, feature_id: str, replaced_by: Optional[str] = None) -> bool:
    p = os.path.join(project_root, MANIFEST_PATH)
    with file_lock(p):
        m = read_manifest(project_root)
        for f in m["features"]:
            if f.get("id") == feature_id:
                f["status"] = "deprecated"
                if replaced_by:
                    f["replaced_by"] = replaced_by
                write_manifest(project_root, m)
                return True
    return False


def check_manifest(project_root: str) -> List[str]:
    warnings: List[str] = []
    for f in read_manifest(project_root)["features"]:
        if f.get("status") == "deprecated":
            continue
        for file in f.get("files", []):
            if not os.path.exists(os.path.join(project_root, file)):
                warnings.append(f'{f["id"]}: "{file}" no longer exists on disk (stale entry)')
    return warnings


def status_icon(status: str) -> str:
    return "+" if status == "implemented" else "~" if status == "partial" else "x"


def manifest_summary(manifest: Dict[str, Any]) -> str:
    feats = manifest.get("features") or []
    if not feats:
        return "No implementation history yet."
    lines = []
    for f in list(reversed(feats[-15:])):
        files = f.get("files") or []
        short = ", ".join(files[:3])
        more = f" +{len(files) - 3} more" if len(files) > 3 else ""
        lines.append(f"- [{status_icon(f.get('status', ''))}] {f.get('id')} — {f.get('summary')} ({short}{more})")
    return "\n".join(lines)


def topic_to_feature_id(topic: str) -> str:
    s = re.sub(r"[^a-z0-9\s-]", "", topic.lower()).strip()
    s = re.sub(r"\s+", "-", s)[:40]
    return re.sub(r"-$", "", s)


def feature_summary(session_path: str, topic: str) -> str:
    p = os.path.join(session_path, "decisions.md")
    try:
        lines = [l for l in read_text(p).split("\n")
                 if l.strip() and not l.startswith("#") and not l.startswith("---")]
        first = lines[0].strip() if lines else ""
        if len(first) > 10:
            return first[:137] + "..." if len(first) > 140 else first
    except OSError:
        pass
    return topic[:137] + "..." if len(topic) > 140 else topic
