"""``roundtable apply`` — the lead knight turns the consensus into edits (spec: README.md:105-108,
200-206,295-311; TODO.md:26,81-142; architecture-docs.md:83,215-218; the command itself is absent
from the reference snapshot, so this is built from those documents).

Pipeline (single attempt, no retry — TODO.md:141):
 1. load the session (latest or ``--session``); it must have reached consensus;
 2. scope = ``status.json`` ``allowed_files`` (``NEW:`` = may be created); sessions without
    scope data are not enforced;
 3. source-context injection: every in-scope existing file with its sha256, truncated at
    80 KB per file / 500 KB total, plus its BLOCK_MAP, and the "EDIT, DON'T REWRITE" rules;
 4. the lead knight (engine-hosted) generates RTDIFF/1 (or ``--response-file`` for tests);
 5. validate: grammar, scope (blocked unless ``--override-scope`` + YES + reason, logged as an
    ``override_scope`` decree), unchanged sha256, block addressing, syntax of the result;
 6. parley (default: confirm per file) / ``--noparley`` (write all) / ``--dry-run`` (write nothing);
 7. backups under ``.roundtable/backups/<session>/`` before any write; status ``applying`` ->
    ``completed``; manifest entry ``implemented`` or ``partial`` (+ ``files_skipped``).
"""
from __future__ import annotations

import difflib
import hashlib
import os
import shutil
from typing import Dict, List, Optional, Tuple

from .. import store
from ..config import load_config
from ..errors import SessionError, ValidationError
from ..utils.atomic import atomic_write_text, read_text
from ..utils.clock import iso_now
from ..utils.ui import UI
from . import rtdiff
from .blocks import block_map

MAX_TOTAL = 500 * 1024
MAX_FILE = 80 * 1024

EDIT_RULES = """REGELS VOOR HET BEWERKEN (VERPLICHT — EDIT, DON'T REWRITE):
1. Antwoord UITSLUITEND met een RTDIFF/1 blok; geen uitleg erbuiten.
2. Adresseer code met de block-ids uit de BLOCK_MAP (of lines:A-B); herschrijf nooit een heel bestand.
3. BLOCK_REPLACE bevat de volledige nieuwe tekst van dat blok, inclusief signatuur.
4. Raak alleen bestanden binnen de scope aan; nieuwe bestanden alleen als FILE: NEW:pad + CREATE.
5. Operaties binnen een bestand mogen elkaar niet overlappen.
6. Behoud bestaande stijl, imports en inspringing; laat ongewijzigde code staan.
7. Het resultaat moet direct compileren / parsen."""

GRAMMAR = """RTDIFF/1
FILE: pad/naar/bestand
BLOCK_REPLACE <block-id>
<<<
nieuwe tekst
>>>
BLOCK_INSERT_AFTER <block-id>
<<<
tekst
>>>
BLOCK_DELETE <block-id>
FILE: NEW:pad/nieuw/bestand
CREATE
<<<
volledige inhoud
>>>
END"""


def sha256(text: str) -> str:
    return hashlib.sha256(text.encode("utf-8")).hexdigest()


def inside_project(root: str, rel: str) -> bool:
    """A knight-proposed path stays inside the project: relative, no '..' escape, no symlink
    escape (checked on the resolved path). Applies even when no scope was recorded, and even
    with --override-scope (which widens the scope, never the project)."""
    if not rel or os.path.isabs(rel) or rel.startswith("~"):
        return False
    base = os.path.realpath(root)
    full = os.path.realpath(os.path.join(base, rel))
    return full != base and full.startswith(base + os.sep)


def scope_sets(allowed: Optional[List[str]]) -> Tuple[Optional[set], set]:
    if allowed is None:
        return None, set()
    existing, new = set(), set()
    for f in allowed:
        if f.upper().startswith("NEW:"):
            new.add(f[4:])
        else:
            existing.add(f)
    return existing | new, new


def source_context(root: str, files: List[str]) -> Tuple[str, Dict[str, str]]:
    """In-scope sources with sha256 + BLOCK_MAP, 80 KB/file, 500 KB total (TODO.md:89-93,122)."""
    parts, hashes, total = [], {}, 0
    for f in files:
        p = os.path.join(root, f)
        if not os.path.isfile(p):
            continue
        text = read_text(p)
        hashes[f] = sha256(text)
        body = text if len(text) <= MAX_FILE else text[:MAX_FILE] + "\n...(truncated at 80KB)"
        if total + len(body) > MAX_TOTAL:
            parts.append(f"### {f} (sha256 {hashes[f]})\n(skipped: 500KB source budget exhausted)")
            continue
        total += len(body)
        numbered = "\n".join(f"{i + 1:5d}| {l}" for i, l in enumerate(body.split("\n")))
        parts.append(f"### {f} (sha256 {hashes[f]})\n{block_map(f, text)}\n```\n{numbered}\n```")
    return "\n\n".join(parts), hashes


def build_apply_prompt(topic: str, decision: str, lead: str, allowed: Optional[List[str]], src: str) -> str:
    scope = "\n".join(f"- {f}" for f in allowed) if allowed else "(geen scope vastgelegd — alle paden toegestaan)"
    return "\n\n".join([
        f"Je bent {lead}, de Lead Knight. De tafel heeft consensus bereikt; jij voert het besluit uit.",
        f"ONDERWERP:\n{topic}", f"BESLUIT:\n{decision}", f"SCOPE (toegestane bestanden):\n{scope}",
        EDIT_RULES, f"FORMAAT:\n{GRAMMAR}", f"BRONCODE:\n{src or '(geen bestaande bestanden in scope)'}",
        "Geef nu je RTDIFF/1:"])


def _diff(path: str, old: Optional[str], new: str) -> str:
    return "".join(difflib.unified_diff((old or "").splitlines(True), new.splitlines(True),
                                        fromfile=f"a/{path}" if old is not None else "/dev/null",
                                        tofile=f"b/{path}"))


def _session(root: str, name: Optional[str]):
    if name:
        path = name if os.path.isabs(name) else os.path.join(root, ".roundtable", "sessions", name)
        if not os.path.isdir(path):
            raise SessionError(f"Session not found: {name}")
        st = store.read_status(path) or {}
        topic = read_text(os.path.join(path, "topic.md")).split("\n\n", 1)[-1].strip()
        return path, st, topic
    s = store.find_latest_session(root)
    if s is None:
        raise SessionError("No sessions found.", hint='Run `roundtable discuss "topic"` first.')
    return s.path, s.status or {}, s.topic or ""


def _generate(root: str, config, lead: str, prompt: str, args, ui: UI) -> str:
    if args.response_file:
        return read_text(args.response_file)
    from ..cli import make_backends
    knight = next((k for k in config.knights if k.name == lead), None) or sorted(config.knights, key=lambda k: k.priority)[0]
    backends, _ = make_backends(config, ui, args, only_knight=knight.name)
    backend = backends.get(knight.adapter)
    if backend is None:
        raise ValidationError(f"lead knight {lead} has no usable backend ({knight.adapter})")
    from ..knights.base import TurnRequest
    ui.dim(f"  {lead} sharpens the quill...")
    res = backend.execute_many([TurnRequest(f"apply:{lead}", prompt, 0, args.max_new_tokens or 2048)],
                               float(config.rules.timeout_per_turn_seconds))[0]
    if isinstance(res, BaseException):
        raise res
    return res.text


def apply_command(args, ui: UI) -> int:
    root = os.getcwd()
    config = load_config(root)
    path, st, topic = _session(root, getattr(args, "session", None))
    if not st.get("consensus_reached"):
        raise SessionError("The latest session has no consensus to apply.",
                           hint="Reach consensus (or let the King choose) before `roundtable apply`.")
    decisions = os.path.join(path, "decisions.md")
    decision = read_text(decisions) if os.path.exists(decisions) else ""
    allowed = st.get("allowed_files")
    scope, new_ok = scope_sets(allowed)
    lead = st.get("lead_knight") or sorted(config.knights, key=lambda k: k.priority)[0].name
    existing = [f for f in (allowed or []) if not f.upper().startswith("NEW:")]
    src, hashes = source_context(root, existing)
    prompt = build_apply_prompt(topic, decision, lead, allowed, src)
    dry = bool(args.dry_run)
    from ..cli import is_writer
    if not dry and is_writer():
        store.update_status(path, phase="applying")
    ui.print(f"\n  Lead Knight {lead} applies the decision{' (dry run)' if dry else ''}.\n", "bold")
    out = _generate(root, config, lead, prompt, args, ui)
    if not is_writer():        # SPMD: the other ranks only took part in the lead knight's decode
        return 0
    edits, warnings = rtdiff.parse(out)
    for w in warnings:
        ui.warn(f"  Warning: {w}")

    override_reason = None
    blocked = [fe.path for fe in edits if scope is not None and fe.path not in scope]
    if blocked:
        for b in blocked:
            ui.error(f"  ✗ {b} is outside the agreed scope")
        if args.override_scope:
            reason = args.reason
            if reason is None:
                from ..cli import ask
                if ask(ui, "  Type YES to override the scope:", "") != "YES":
                    raise ValidationError("scope override not confirmed")
                reason = ask(ui, "  Reason for the override:", "")
            if not reason:
                raise ValidationError("--override-scope requires a reason")
            override_reason = reason
            if not dry:
                store.add_decree_entry(root, "override_scope", os.path.basename(path), topic, reason)
        else:
            ui.dim("  (use --override-scope to write them anyway)")

    plan: List[Tuple[str, Optional[str], str]] = []
    skipped: List[str] = []
    for fe in edits:
        if not inside_project(root, fe.path):
            ui.error(f"  ✗ {fe.path} is outside the project (absolute or '..' path) — never written")
            skipped.append(fe.path)
            continue
        if fe.path in blocked and override_reason is None:
            skipped.append(fe.path)
            continue
        full = os.path.join(root, fe.path)
        old = read_text(full) if os.path.isfile(full) else None
        if fe.path in hashes and old is not None and sha256(old) != hashes[fe.path]:
            ui.error(f"  ✗ {fe.path} changed on disk since the knight read it (sha256 mismatch)")
            skipped.append(fe.path)
            continue
        if old is None and scope is not None and fe.path not in new_ok and override_reason is None:
            ui.error(f"  ✗ {fe.path} does not exist and is not declared NEW: in the scope")
            skipped.append(fe.path)
            continue
        try:
            new = rtdiff.apply_edit(fe, old)
        except ValidationError as e:
            ui.error(f"  ✗ {e.message}")
            skipped.append(fe.path)
            continue
        err = rtdiff.validate_syntax(fe.path, new)
        if err:
            ui.error(f"  ✗ validation failed: {err}")
            skipped.append(fe.path)
            continue
        plan.append((fe.path, old, new))

    written: List[str] = []
    backup_dir = os.path.join(root, ".roundtable", "backups", os.path.basename(path))
    for rel, old, new in plan:
        ui.print(f"\n  {'+' if old is None else '~'} {rel}", "cyan")
        ui.print(_diff(rel, old, new) or "  (no change)")
        if dry:
            continue
        if not args.noparley and not args.yes:
            from ..cli import confirm
            if not confirm(ui, f"  Write {rel}?", True):
                skipped.append(rel)
                continue
        full = os.path.join(root, rel)
        if old is not None:
            bpath = os.path.join(backup_dir, rel + ".bak")
            os.makedirs(os.path.dirname(bpath), exist_ok=True)
            shutil.copy2(full, bpath)
        atomic_write_text(full, new)
        written.append(rel)

    if dry:
        # the plan is kept with the session (never in the project tree): review it, then apply for real
        import json as _json
        atomic_write_text(os.path.join(path, "apply-plan.json"), _json.dumps({
            "lead_knight": lead, "created_at": iso_now(),
            "planned": [{"path": rel, "new_file": old is None, "diff": _diff(rel, old, new)} for rel, old, new in plan],
            "skipped": skipped}, indent=2, ensure_ascii=False) + "\n")
        ui.ok(f"\n  Dry run complete: {len(plan)} file(s) would be written, {len(skipped)} skipped. Nothing was written.")
        return 0
    if not plan and not written:
        store.update_status(path, phase="consensus_reached")
        raise ValidationError("Nothing could be applied — every edit failed validation or scope.",
                              hint="Read decisions.md and apply manually, or re-run apply.")
    status = "implemented" if not skipped else "partial"
    entry = {"id": store.topic_to_feature_id(topic) or os.path.basename(path), "session": os.path.basename(path),
             "status": status, "files": written, "summary": store.feature_summary(path, topic),
             "applied_at": iso_now(), "lead_knight": lead}
    if skipped:
        entry["files_skipped"] = skipped
    store.add_manifest_entry(root, entry)
    store.update_status(path, phase="completed")
    ui.ok(f"\n  The deed is done: {len(written)} file(s) written ({status}).")
    return 0
