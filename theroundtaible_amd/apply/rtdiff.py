"""RTDIFF/1 — block-level edit format for ``roundtable apply`` (grammar defined here; TODO.md:87,128-137).

    RTDIFF/1
    FILE: src/server.ts
    BLOCK_REPLACE function:handleRequest
    <<<
    ...new text of the whole block...
    >>>
    BLOCK_INSERT_AFTER class:Cache
    <<<
    ...text inserted after the block's last line...
    >>>
    BLOCK_DELETE lines:40-52
    FILE: NEW:src/cache/policy.ts
    CREATE
    <<<
    ...full content of the new file...
    >>>
    END

* ops may be written with or without a colon after the keyword (``BLOCK_DELETE: id``);
* every op addresses blocks of the file *as it was read* (the sha256 in the prompt);
  ops on one file must not overlap and are applied bottom-up;
* the legacy search/replace form is still accepted, with a deprecation warning::

    EDIT: path
    <<<<<<< SEARCH
    old text
    =======
    new text
    >>>>>>> REPLACE
"""
from __future__ import annotations

import ast
import json
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from ..errors import ValidationError
from .blocks import BRACE_EXTS, resolve, scan

OPS = ("BLOCK_REPLACE", "BLOCK_INSERT_AFTER", "BLOCK_DELETE", "CREATE")


@dataclass
class Op:
    kind: str
    target: str = ""          # block id (empty for CREATE / EDIT)
    body: str = ""
    search: str = ""          # legacy EDIT


@dataclass
class FileEdit:
    path: str
    is_new: bool = False
    ops: List[Op] = field(default_factory=list)
    legacy: bool = False


def _norm_path(p: str) -> Tuple[str, bool]:
    p = p.strip().strip("`").strip()
    new = p.upper().startswith("NEW:")
    if new:
        p = p[4:].strip()
    p = p.replace("\\", "/")
    if p.startswith("./"):
        p = p[2:]
    return p, new


def parse(text: str) -> Tuple[List[FileEdit], List[str]]:
    """Parse knight output into per-file edits. Returns (edits, warnings)."""
    warnings: List[str] = []
    edits: List[FileEdit] = []
    start = text.find("RTDIFF/1")
    if start >= 0:
        lines = text[start:].split("\n")[1:]
        edits.extend(_parse_rtdiff(lines))
    legacy = _parse_legacy(text)
    if legacy:
        warnings.append("legacy EDIT: search/replace blocks are deprecated — use RTDIFF/1 BLOCK_* operations")
        edits.extend(legacy)
    if not edits:
        raise ValidationError("no RTDIFF/1 or EDIT: blocks found in the lead knight's output")
    return edits, warnings


def _parse_rtdiff(lines: List[str]) -> List[FileEdit]:
    edits: List[FileEdit] = []
    cur: Optional[FileEdit] = None
    i = 0
    while i < len(lines):
        raw = lines[i]
        line = raw.strip()
        i += 1
        if not line or line.startswith("```"):
            continue
        if line == "END":
            break
        if line.startswith("FILE:"):
            path, new = _norm_path(line[5:])
            cur = FileEdit(path, new)
            edits.append(cur)
            continue
        m = re.match(r"^(BLOCK_REPLACE|BLOCK_INSERT_AFTER|BLOCK_DELETE|CREATE)\s*:?\s*(.*)$", line)
        if not m:
            raise ValidationError(f"RTDIFF/1: unexpected line {i}: {raw!r}")
        if cur is None:
            raise ValidationError(f"RTDIFF/1: operation before any FILE: (line {i})")
        kind, target = m.group(1), m.group(2).strip()
        op = Op(kind, target)
        if kind in ("BLOCK_REPLACE", "BLOCK_INSERT_AFTER", "CREATE"):
            while i < len(lines) and not lines[i].strip():
                i += 1
            if i >= len(lines) or lines[i].strip() != "<<<":
                raise ValidationError(f"RTDIFF/1: {kind} {target} needs a <<< ... >>> body (line {i + 1})")
            i += 1
            body: List[str] = []
            while i < len(lines) and lines[i].strip() != ">>>":
                body.append(lines[i])
                i += 1
            if i >= len(lines):
                raise ValidationError(f"RTDIFF/1: unterminated body for {kind} {target}")
            i += 1
            op.body = "\n".join(body)
        elif not target:
            raise ValidationError("RTDIFF/1: BLOCK_DELETE needs a block id")
        cur.ops.append(op)
    return edits


_LEGACY = re.compile(r"EDIT:\s*(\S+)\s*\n<<<<<<< SEARCH\n([\s\S]*?)\n=======\n([\s\S]*?)\n>>>>>>> REPLACE")


def _parse_legacy(text: str) -> List[FileEdit]:
    out: Dict[str, FileEdit] = {}
    for m in _LEGACY.finditer(text):
        path, _ = _norm_path(m.group(1))
        fe = out.setdefault(path, FileEdit(path, legacy=True))
        fe.ops.append(Op("EDIT", search=m.group(2), body=m.group(3)))
    return list(out.values())


def apply_edit(fe: FileEdit, original: Optional[str]) -> str:
    """Return the new content of one file (raises ValidationError on any addressing problem)."""
    if any(op.kind == "CREATE" for op in fe.ops):
        if original is not None and not fe.is_new:
            raise ValidationError(f"{fe.path}: CREATE on an existing file (mark it NEW: only for new files)")
        if len(fe.ops) != 1:
            raise ValidationError(f"{fe.path}: CREATE must be the only operation on a file")
        body = fe.ops[0].body
        return body if body.endswith("\n") else body + "\n"
    if original is None:
        raise ValidationError(f"{fe.path}: file does not exist (use FILE: NEW:{fe.path} + CREATE)")
    if fe.legacy:
        text = original
        for op in fe.ops:
            n = text.count(op.search)
            if n != 1:
                raise ValidationError(f"{fe.path}: EDIT search text found {n} times (must be exactly once)")
            text = text.replace(op.search, op.body, 1)
        return text
    lines = original.split("\n")
    blocks = scan(fe.path, original)
    spans = []
    for op in fe.ops:
        rng = resolve(op.target, blocks, len(lines))
        if rng is None:
            raise ValidationError(f"{fe.path}: unknown block '{op.target}' (see BLOCK_MAP)")
        spans.append((rng, op))
    # overlap check on the original addressing (INSERT_AFTER occupies a zero-width point after its end)
    occupied = sorted(((a, b if op.kind != "BLOCK_INSERT_AFTER" else a - 1, op) for (a, b), op in spans
                       if op.kind != "BLOCK_INSERT_AFTER"), key=lambda t: t[0])
    for (a1, b1, o1), (a2, b2, o2) in zip(occupied, occupied[1:]):
        if a2 <= b1:
            raise ValidationError(f"{fe.path}: operations on '{o1.target}' and '{o2.target}' overlap")
    for (a, b), op in sorted(spans, key=lambda s: (s[0][1], s[1].kind == "BLOCK_INSERT_AFTER"), reverse=True):
        body = op.body.split("\n") if op.body else []
        if op.kind == "BLOCK_REPLACE":
            lines[a - 1:b] = body
        elif op.kind == "BLOCK_DELETE":
            del lines[a - 1:b]
        elif op.kind == "BLOCK_INSERT_AFTER":
            lines[b:b] = body
    return "\n".join(lines)


def validate_syntax(path: str, text: str) -> Optional[str]:
    """None if the result parses for its language (Python: ast; JSON; brace languages: balanced)."""
    if path.endswith(".py"):
        try:
            ast.parse(text)
        except SyntaxError as e:
            return f"{path}: Python syntax error at line {e.lineno}: {e.msg}"
    elif path.endswith(".json"):
        try:
            json.loads(text)
        except ValueError as e:
            return f"{path}: invalid JSON: {e}"
    elif path.endswith(BRACE_EXTS):
        bal = _brace_balance(text)
        if bal != 0:
            return f"{path}: unbalanced braces ({bal:+d})"
    return None


def _brace_balance(text: str) -> int:
    depth = 0
    in_str = None
    block = False
    i = 0
    while i < len(text):
        c = text[i]
        n = text[i + 1] if i + 1 < len(text) else ""
        if block:
            if c == "*" and n == "/":
                block = False
                i += 1
        elif in_str:
            if c == "\\":
                i += 1
            elif c == in_str or (c == "\n" and in_str != "`"):
                in_str = None
        elif c == "/" and n == "/":
            j = text.find("\n", i)
            i = len(text) if j < 0 else j
            continue
        elif c == "/" and n == "*":
            block = True
            i += 1
        elif c in "'\"`":
            in_str = c
        elif c in "{([":
            depth += 1
        elif c in "})]":
            depth -= 1
        i += 1
    return depth
