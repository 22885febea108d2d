"""Block scanner: named, line-addressed code blocks for RTDIFF/1 (TODO.md:87,128-137).

The reference's block scanner is not in the snapshot; this is our own design. A block is
``(id, kind, start_line, end_line)`` with 1-based inclusive lines. Ids are stable,
human-readable addresses the lead knight uses instead of rewriting files:

* Python (via ``ast``, exact): ``def:name``, ``class:Name``, ``def:Class.method``;
* brace languages (ts/tsx/js/jsx/java/go/rs/c/cpp/hip): ``function:name``,
  ``class:Name``, ``method:Class.name``, ``const:name`` (arrow functions / objects),
  ``interface:Name``/``type:Name``/``enum:Name``; ends found by a string/comment-aware
  brace matcher;
* always available: ``lines:a-b`` (any 1-based inclusive range) and ``file`` (whole file).

The BLOCK_MAP shown to the knight lists the scanned ids with their line ranges.
"""
from __future__ import annotations

import ast
import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple


@dataclass(frozen=True)
class Block:
    id: str
    kind: str
    start: int   # 1-based inclusive
    end: int     # 1-based inclusive


BRACE_EXTS = (".ts", ".tsx", ".js", ".jsx", ".mjs", ".cjs", ".java", ".go", ".rs", ".c", ".cc", ".cpp", ".h",
              ".hpp", ".hip", ".cu", ".cs", ".kt", ".swift")


def scan(path: str, text: str) -> List[Block]:
    if path.endswith(".py"):
        return _scan_python(text)
    if path.endswith(BRACE_EXTS):
        return _scan_braces(text)
    return []


def _scan_python(text: str) -> List[Block]:
    try:
        tree = ast.parse(text)
    except SyntaxError:
        return []
    out: List[Block] = []

    def start_of(node) -> int:
        decos = getattr(node, "decorator_list", [])
        return min([node.lineno] + [d.lineno for d in decos])

    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            out.append(Block(f"def:{node.name}", "function", start_of(node), node.end_lineno))
        elif isinstance(node, ast.ClassDef):
            out.append(Block(f"class:{node.name}", "class", start_of(node), node.end_lineno))
            for sub in node.body:
                if isinstance(sub, (ast.FunctionDef, ast.AsyncFunctionDef)):
                    out.append(Block(f"def:{node.name}.{sub.name}", "method", start_of(sub), sub.end_lineno))
    return out


_DECL = [
    ("function", re.compile(r"^\s*(?:export\s+)?(?:default\s+)?(?:async\s+)?function\*?\s+([A-Za-z_$][\w$]*)\s*[<(]")),
    ("class", re.compile(r"^\s*(?:export\s+)?(?:default\s+)?(?:abstract\s+)?class\s+([A-Za-z_$][\w$]*)")),
    ("interface", re.compile(r"^\s*(?:export\s+)?interface\s+([A-Za-z_$][\w$]*)")),
    ("enum", re.compile(r"^\s*(?:export\s+)?(?:const\s+)?enum\s+([A-Za-z_$][\w$]*)")),
    ("type", re.compile(r"^\s*(?:export\s+)?type\s+([A-Za-z_$][\w$]*)\s*(?:<[^=]*>)?\s*=\s*\{")),
    ("const", re.compile(r"^\s*(?:export\s+)?(?:const|let|var)\s+([A-Za-z_$][\w$]*)\s*(?::[^=]+)?=\s*"
                         r"(?:async\s*)?(?:\([^)]*\)|[A-Za-z_$][\w$]*)?\s*(?:=>)?\s*\{")),
]
_METHOD = re.compile(r"^\s*(?:public\s+|private\s+|protected\s+|static\s+|async\s+|override\s+|readonly\s+)*"
                     r"(?:get\s+|set\s+)?([A-Za-z_$][\w$]*)\s*(?:<[^>]*>)?\s*\([^;]*\)\s*(?::[^{;]+)?\{\s*$")
_KEYWORDS = {"if", "for", "while", "switch", "catch", "function", "return", "else", "do", "try", "with"}


def _brace_end(lines: List[str], start_idx: int) -> Optional[int]:
    """Index of the line where the first '{' at/after start_idx is closed (string/comment aware)."""
    depth = 0
    seen = False
    in_str: Optional[str] = None
    block_comment = False
    for i in range(start_idx, len(lines)):
        line = lines[i]
        j = 0
        while j < len(line):
            c = line[j]
            nxt = line[j + 1] if j + 1 < len(line) else ""
            if block_comment:
                if c == "*" and nxt == "/":
                    block_comment = False
                    j += 1
            elif in_str:
                if c == "\\":
                    j += 1
                elif c == in_str:
                    in_str = None
            elif c == "/" and nxt == "/":
                break
            elif c == "/" and nxt == "*":
                block_comment = True
                j += 1
            elif c in ("'", '"', "`"):
                in_str = c
            elif c == "{":
                depth += 1
                seen = True
            elif c == "}":
                depth -= 1
                if seen and depth == 0:
                    return i
            j += 1
        if in_str in ("'", '"'):
            in_str = None  # unterminated single-line string: recover
    return None


def _scan_braces(text: str) -> List[Block]:
    lines = text.split("\n")
    out: List[Block] = []
    i = 0
    while i < len(lines):
        line = lines[i]
        hit = None
        for kind, pat in _DECL:
            m = pat.match(line)
            if m:
                hit = (kind, m.group(1))
                break
        if hit:
            end = _brace_end(lines, i)
            if end is not None:
                kind, name = hit
                out.append(Block(f"{kind}:{name}", kind, i + 1, end + 1))
                if kind == "class":
                    out.extend(_scan_methods(lines, i + 1, end, name))
                i = end + 1
                continue
        i += 1
    return out


def _scan_methods(lines: List[str], lo: int, hi: int, cls: str) -> List[Block]:
    out = []
    i = lo
    while i < hi:
        m = _METHOD.match(lines[i])
        if m and m.group(1) not in _KEYWORDS:
            end = _brace_end(lines, i)
            if end is not None and end <= hi:
                out.append(Block(f"method:{cls}.{m.group(1)}", "method", i + 1, end + 1))
                i = end + 1
                continue
        i += 1
    return out


def resolve(block_id: str, blocks: List[Block], n_lines: int) -> Optional[Tuple[int, int]]:
    """Line range (1-based inclusive) addressed by ``block_id``, or None if unknown."""
    if block_id == "file":
        return (1, n_lines)
    m = re.fullmatch(r"lines:(\d+)-(\d+)", block_id)
    if m:
        a, b = int(m.group(1)), int(m.group(2))
        return (a, b) if 1 <= a <= b <= n_lines else None
    for b in blocks:
        if b.id == block_id:
            return (b.start, b.end)
    return None


def block_map(path: str, text: str) -> str:
    blocks = scan(path, text)
    n = len(text.split("\n"))
    lines = [f"  {b.id}  (lines {b.start}-{b.end})" for b in blocks]
    lines.append(f"  lines:A-B  (any range within 1-{n})")
    return f"BLOCK_MAP {path}:\n" + "\n".join(lines)
