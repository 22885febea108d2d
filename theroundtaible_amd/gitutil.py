"""Git helpers (`src/utils/git.ts:6-41`): every call returns None on failure."""
from __future__ import annotations

import subprocess
from typing import List, Optional


def _git(args: List[str], cwd: Optional[str]) -> Optional[str]:
    try:
        r = subprocess.run(["git"] + args, cwd=cwd, capture_output=True, text=True, timeout=30)
    except (OSError, subprocess.SubprocessError):
        return None
    if r.returncode != 0:
        return None
    return r.stdout


def git_branch(cwd: Optional[str] = None) -> Optional[str]:
    out = _git(["rev-parse", "--abbrev-ref", "HEAD"], cwd)
    return out.strip() if out is not None else None


def git_diff(cwd: Optional[str] = None) -> Optional[str]:
    """Staged + unstaged diff, staged first (git.ts:18-29)."""
    staged = _git(["diff", "--cached"], cwd)
    if staged is None:
        return None
    unstaged = _git(["diff"], cwd)
    if unstaged is None:
        return None
    # execa strips the trailing newline of stdout; mirror that before joining.
    parts = [p.rstrip("\n") for p in (staged, unstaged) if p.rstrip("\n")]
    combined = "\n".join(parts)
    return combined or None


def recent_commits(n: int = 5, cwd: Optional[str] = None) -> Optional[str]:
    out = _git(["log", "--oneline", f"-{n}"], cwd)
    if out is None:
        return None
    return out.strip() or None
