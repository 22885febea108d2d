"""Project context gathering (`src/utils/context.ts:12-187`).

Budgets are the reference's: key files <= 5 x 2,000 chars, source
files <= 30 with a character budget (default 200,000, or the smallest budget any
seated knight reports — the engine reports one from its KV/context capacity).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, List, Optional

from .gitutil import git_branch, git_diff, recent_commits
from .prompt import TurnContext
from .store.chronicle import read_chronicle

KEY_PATTERNS = ("package.json", "tsconfig.json", "README.md", "CLAUDE.md")
SOURCE_EXTS = (".ts", ".tsx", ".js", ".jsx", ".py", ".rs", ".go", ".java", ".json")
SOURCE_EXCLUDE = ("package-lock.json", "yarn.lock", "pnpm-lock.yaml", "bun.lockb", ".env", ".env.local")


def _ignored(rel: str, name: str, patterns: List[str]) -> bool:
    return any(rel.startswith(p) or name == p or f"/{p}/" in rel or f"\\{p}\\" in rel for p in patterns)


def project_files(root: str, ignore: List[str]) -> List[str]:
    """Depth-first walk in directory-listing order, skipping ignore patterns (context.ts:12-46)."""
    out: List[str] = []

    def walk(d: str) -> None:
        try:
            entries = sorted(os.scandir(d), key=lambda e: e.name)
        except OSError:
            return
        for e in entries:
            rel = os.path.relpath(e.path, root)
            if _ignored(rel, e.name, ignore):
                continue
            if e.is_dir(follow_symlinks=False):
                walk(e.path)
            elif e.is_file(follow_symlinks=False):
                out.append(rel)

    walk(root)
    return out


def read_key_files(root: str, files: List[str]) -> str:
    chunks = []
    for f in [f for f in files if any(f.endswith(p) for p in KEY_PATTERNS)][:5]:
        try:
            with open(os.path.join(root, f), "r", encoding="utf-8", errors="replace") as fh:
                c = fh.read()
        except OSError:
            continue
        if len(c) > 2000:
            c = c[:2000] + "\n...(truncated)"
        chunks.append(f"### {f}\n```\n{c}\n```")
    return "\n\n".join(chunks)


def read_source_files(root: str, ignore: List[str], max_chars: int = 50000,
                      warn: Optional[Callable[[str], None]] = None) -> str:
    files = [f for f in project_files(root, ignore)
             if f.endswith(SOURCE_EXTS) and not f.endswith(SOURCE_EXCLUDE)][:30]
    chunks, total, skipped = [], 0, 0
    for f in files:
        if total >= max_chars:
            skipped += 1
            continue
        try:
            with open(os.path.join(root, f), "r", encoding="utf-8", errors="replace") as fh:
                c = fh.read()
        except OSError:
            continue
        t = c[:min(len(c), max_chars - total)]
        chunks.append(f"### {f}\n```\n{t}\n```")
        total += len(t)
    if skipped and warn:
        warn(f"  The scrolls overflow! {skipped} file(s) skipped — the knights can only carry "
             f"{round(max_chars / 1024)}KB into battle.")
    return "\n\n".join(chunks)


def build_context(root: str, topic: str, ignore: List[str], chronicle_path: str,
                  read_source: bool = False, max_source_chars: int = 200_000,
                  warn: Optional[Callable[[str], None]] = None) -> TurnContext:
    with ThreadPoolExecutor(max_workers=5) as ex:
        f_chr = ex.submit(read_chronicle, root, chronicle_path)
        f_br = ex.submit(git_branch, root)
        f_diff = ex.submit(git_diff, root)
        f_log = ex.submit(recent_commits, 5, root)
        f_files = ex.submit(project_files, root, ignore)
        files = f_files.result()
        ctx = TurnContext(topic=topic, chronicle=f_chr.result(), git_branch=f_br.result(),
                          git_diff=f_diff.result(), recent_commits=f_log.result())
    ctx.key_file_contents = read_key_files(root, files)
    if read_source:
        ctx.source_file_contents = read_source_files(root, ignore, max_source_chars, warn)
    return ctx
