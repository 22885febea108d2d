"""Consensus engine: pull the structured verdict out of free-form knight output.

Parity map (reference `src/consensus.ts`):
  * :func:`validate_files_to_modify`      consensus.ts:10-49
  * :func:`missing_scope_warning`         consensus.ts:54-65
  * :func:`balanced_objects`              consensus.ts:71-112 (string-aware brace scanner)
  * :func:`parse_consensus`               consensus.ts:118-145 (fenced json, any fence, balanced)
  * :func:`check_consensus`               consensus.ts:217-223 (score only; pending issues informational)
  * :func:`check_negative_consensus`      consensus.ts:230-239 (>=2 blocks, all <= 3)
  * :func:`summarize_consensus`           consensus.ts:244-279
  * :func:`repair_json`                   consensus.ts:287-292

The scanner is a single pass over the text; it is also what the engine's optional
"stop when the consensus JSON closes" decode criterion uses (see
:class:`ConsensusStopDetector`), so host parsing and device-side early exit agree.
"""
from __future__ import annotations

import json
import math
import re
from typing import Any, Iterable, List, Optional

from .types import ConsensusBlock

_FENCED = (
    re.compile(r"```json\s*\n?([\s\S]*?)\n?\s*```"),
    re.compile(r"```\s*\n?([\s\S]*?)\n?\s*```"),
)

_MEANINGLESS = frozenset({
    "", "none", "no", "n/a", "na", "nil", "null", "-",
    "no issues", "no open issues", "no pending issues",
    "geen", "geen issues", "geen open issues",
    "all resolved", "all issues resolved", "resolved",
    "nothing", "no concerns", "no remaining issues",
})


def _js_truthy(v: Any) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0 and not (isinstance(v, float) and math.isnan(v))
    if isinstance(v, str):
        return v != ""
    return True


def _is_js_number(v: Any) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def validate_files_to_modify(raw: Any) -> List[str]:
    """Normalize a ``files_to_modify`` list: relative, forward slashes, no '..', deduped, ``NEW:`` kept."""
    if not isinstance(raw, list):
        return []
    seen = set()
    out: List[str] = []
    for item in raw:
        if not isinstance(item, str):
            continue
        path = item.strip()
        if not path:
            continue
        is_new = path.upper().startswith("NEW:")
        if is_new:
            path = path[4:].strip()
        path = path.replace("\\", "/")
        if path.startswith("./"):
            path = path[2:]
        if path.startswith("/") or ".." in path or not path:
            continue
        norm = f"NEW:{path}" if is_new else path
        if norm in seen:
            continue
        seen.add(norm)
        out.append(norm)
    return out


def missing_scope_warning(block: ConsensusBlock) -> Optional[str]:
    if block.consensus_score >= 9 and not block.files_to_modify:
        return (f"  Warning: {block.knight} agreed (score {block.consensus_score}) but didn't "
                f"specify files_to_modify. Scope enforcement will be skipped for this knight.")
    return None


def balanced_objects(text: str, key: str) -> List[str]:
    """Every top-level ``{...}`` object in *text* (string/escape aware) that mentions ``"key"``."""
    token = f'"{key}"'
    found: List[str] = []
    depth = 0
    start = -1
    in_str = False
    esc = False
    for i, ch in enumerate(text):
        if in_str:
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
            continue
        if ch == '"':
            in_str = True
        elif ch == "{":
            if depth == 0:
                start = i
            depth += 1
        elif ch == "}" and depth > 0:
            depth -= 1
            if depth == 0 and start >= 0:
                cand = text[start:i + 1]
                if token in cand:
                    found.append(cand)
                start = -1
    return found


def repair_json(raw: str) -> str:
    """Local-model JSON repair: drop ``//`` comments, trailing commas, single quotes -> double."""
    out = re.sub(r"//[^\n]*", "", raw)
    out = re.sub(r",\s*([}\]])", r"\1", out)
    return out.replace("'", '"')


def _reject_constant(name: str):  # JSON.parse rejects NaN/Infinity
    raise ValueError(name)


def _sanitize_pending(raw: Any) -> List[str]:
    if not isinstance(raw, list):
        return []
    items = [s.strip() for s in raw if isinstance(s, str)]
    return [s for s in items if s.lower() not in _MEANINGLESS]


def _block_from_json(text: str, knight: str, rnd: int) -> Optional[ConsensusBlock]:
    try:
        obj = json.loads(text, parse_constant=_reject_constant)
    except (ValueError, RecursionError):
        return None
    if not isinstance(obj, dict) or not _is_js_number(obj.get("consensus_score")):
        return None
    fr = obj.get("file_requests")
    vc = obj.get("verify_commands")
    aw = obj.get("agrees_with")
    return ConsensusBlock(
        knight=obj["knight"] if _js_truthy(obj.get("knight")) else knight,
        round=obj["round"] if _js_truthy(obj.get("round")) else rnd,
        consensus_score=obj["consensus_score"],
        agrees_with=list(aw) if isinstance(aw, list) else [],
        pending_issues=_sanitize_pending(obj.get("pending_issues")),
        proposal=obj.get("proposal"),
        files_to_modify=validate_files_to_modify(obj.get("files_to_modify")),
        file_requests=list(fr[:4]) if isinstance(fr, list) else [],
        verify_commands=list(vc[:4]) if isinstance(vc, list) else [],
    )


def _try_parse(text: str, knight: str, rnd: int) -> Optional[ConsensusBlock]:
    for attempt in (text, repair_json(text)):
        blk = _block_from_json(attempt, knight, rnd)
        if blk is not None:
            return blk
    return None


def parse_consensus(response: str, knight: str, rnd: int) -> Optional[ConsensusBlock]:
    """Extract the ConsensusBlock from a knight response, or None if it forgot the rules."""
    for pat in _FENCED:
        m = pat.search(response)
        if not m or not m.group(1):
            continue
        blk = _try_parse(m.group(1).strip(), knight, rnd)
        if blk is not None:
            return blk
    for cand in balanced_objects(response, "consensus_score"):
        blk = _try_parse(cand, knight, rnd)
        if blk is not None:
            return blk
    return None


def check_consensus(blocks: Iterable[ConsensusBlock], threshold: float) -> bool:
    blocks = list(blocks)
    return bool(blocks) and all(b.consensus_score >= threshold for b in blocks)


def check_negative_consensus(blocks: Iterable[ConsensusBlock], rejection_threshold: float = 3) -> bool:
    blocks = list(blocks)
    return len(blocks) >= 2 and all(b.consensus_score <= rejection_threshold for b in blocks)


def _fmt_num(x: float) -> str:
    return str(int(x)) if isinstance(x, float) and x.is_integer() else str(x)


def _join(items: Iterable[Any]) -> str:
    return ", ".join(_js_str(i) for i in items)


def _js_str(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "null"
    if isinstance(v, float):
        return _fmt_num(v)
    if isinstance(v, (dict, list)):
        return "[object Object]" if isinstance(v, dict) else ",".join(_js_str(x) for x in v)
    return str(v)


def summarize_consensus(blocks: List[ConsensusBlock]) -> str:
    if not blocks:
        return "No consensus data yet."
    lines: List[str] = []
    for b in blocks:
        s = b.consensus_score
        status = "AGREES" if s >= 9 else "PARTIAL" if s >= 6 else "DISAGREES"
        lines.append(f"- **{b.knight}** (Round {b.round}): Score {_fmt_num(s)}/10 [{status}]")
        if b.agrees_with:
            lines.append(f"  Agrees with: {_join(b.agrees_with)}")
        if b.pending_issues:
            lines.append(f"  Pending: {_join(b.pending_issues)}")
        if b.files_to_modify:
            lines.append(f"  Scope: {_join(b.files_to_modify)}")
    avg = sum(b.consensus_score for b in blocks) / len(blocks)
    lines.append(f"\nAverage score: {avg:.1f}/10")
    return "\n".join(lines)


def strip_consensus_json(text: str, key: str = "consensus_score") -> str:
    """Display helper (orchestrator.ts:79-108): remove ```json fences and the first bare block with *key*."""
    result = re.sub(r"```json[\s\S]*?```", "", text)
    k = result.find(f'"{key}"')
    if k == -1:
        return result
    open_idx = result.rfind("{", 0, k)
    if open_idx == -1:
        return result
    depth = 0
    for i in range(open_idx, len(result)):
        c = result[i]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return result[:open_idx] + result[i + 1:]
    return result


class ConsensusStopDetector:
    """Incremental detector: True once the text contains a *parseable* consensus block.

    Used by the engine as an optional early-stop criterion (``stop_on_consensus``):
    the decode loop feeds detokenized text chunks and stops a sequence as soon as its
    verdict is complete, instead of burning the rest of ``max_new_tokens``.
    """

    def __init__(self, knight: str = "", rnd: int = 0):
        self.buf: List[str] = []
        self.knight = knight
        self.rnd = rnd
        self._last_len = 0

    def feed(self, chunk: str) -> bool:
        self.buf.append(chunk)
        if "}" not in chunk and "`" not in chunk:
            return False
        text = "".join(self.buf)
        return parse_consensus(text, self.knight, self.rnd) is not None
