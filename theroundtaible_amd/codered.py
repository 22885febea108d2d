"""``roundtable code-red`` — diagnostic mode (spec: README.md:159-175; architecture-docs.md:119-129,151-167).

The reference ships this disabled ("coming in v1.1"); here it is implemented from the spec:

* round 1 **triage**: every doctor (knight) sees the symptoms and gives a first assessment;
* round 2 **blind**: doctors diagnose independently — nobody sees another doctor's round-2
  answer (this is exactly the engine's ``parallel`` round semantics, so all doctors decode as
  one batch);
* rounds 3+ **convergence**: doctors see everything and converge on a root cause.

Each doctor ends with a JSON verdict ``{confidence_score, root_cause_key, evidence, rules_out,
confirms, file_requests, next_test}``. Convergence = at least two doctors share a
``root_cause_key`` (exact, or fuzzy: same normalized token set / one contains the other) with
confidence >= 8. Findings are appended to ``.roundtable/error-log.md`` as ``CR-XXX`` entries
with status OPEN / RESOLVED / PARKED.
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import store
from .config import load_config
from .consensus import balanced_objects, repair_json
from .errors import ConfigError
from .knights.base import TurnRequest
from .tools import resolve_file_requests
from .utils.atomic import atomic_write_text, file_lock, read_text
from .utils.clock import iso_now
from .utils.ui import UI

ERROR_LOG = os.path.join(".roundtable", "error-log.md")
PHASES = {1: "TRIAGE", 2: "BLIND"}


@dataclass
class Diagnosis:
    doctor: str
    round: int
    confidence_score: float
    root_cause_key: str
    evidence: List[str] = field(default_factory=list)
    rules_out: List[str] = field(default_factory=list)
    confirms: List[str] = field(default_factory=list)
    file_requests: List[str] = field(default_factory=list)
    next_test: str = ""


def parse_diagnosis(text: str, doctor: str, rnd: int) -> Optional[Diagnosis]:
    cands = [m.group(1) for m in re.finditer(r"```(?:json)?\s*\n?([\s\S]*?)\n?\s*```", text)]
    cands += balanced_objects(text, "root_cause_key")
    for c in cands:
        for attempt in (c, repair_json(c)):
            try:
                o = json.loads(attempt)
            except ValueError:
                continue
            if isinstance(o, dict) and isinstance(o.get("confidence_score"), (int, float)) \
                    and isinstance(o.get("root_cause_key"), str) and o["root_cause_key"].strip():
                lst = lambda k: [str(x) for x in o.get(k, [])] if isinstance(o.get(k), list) else []  # noqa: E731
                return Diagnosis(doctor, rnd, o["confidence_score"], o["root_cause_key"].strip(), lst("evidence"),
                                 lst("rules_out"), lst("confirms"), lst("file_requests")[:4], str(o.get("next_test", "")))
    return None


def _norm_key(k: str) -> str:
    return re.sub(r"[^a-z0-9]+", "-", k.lower()).strip("-")


def keys_match(a: str, b: str) -> bool:
    na, nb = _norm_key(a), _norm_key(b)
    if na == nb:
        return True
    ta, tb = set(na.split("-")), set(nb.split("-"))
    return bool(ta) and (ta == tb or na in nb or nb in na)


def check_convergence(latest: Dict[str, Diagnosis], min_conf: float = 8) -> Optional[str]:
    confident = [d for d in latest.values() if d.confidence_score >= min_conf]
    for i, a in enumerate(confident):
        for b in confident[i + 1:]:
            if keys_match(a.root_cause_key, b.root_cause_key):
                return a.root_cause_key
    return None


def doctor_prompt(name: str, symptoms: str, rnd: int, visible: List[str], evidence: str) -> str:
    phase = PHASES.get(rnd, "CONVERGENTIE")
    rules = {
        "TRIAGE": "Geef een eerste inschatting van de symptomen en welke bewijzen je nodig hebt.",
        "BLIND": "Stel ONAFHANKELIJK een diagnose: je ziet bewust niet wat de andere doctors nu zeggen.",
        "CONVERGENTIE": "Vergelijk de diagnoses, weerleg of bevestig, en convergeer op de oorzaak.",
    }[phase]
    hist = "\n\n---\n\n".join(visible) if visible else "(nog geen eerdere rondes)"
    return (f"CODE-RED. Je bent Dr. {name}. Fase: {phase} (ronde {rnd}).\n{rules}\n\nSYMPTOMEN:\n{symptoms}\n\n"
            f"EERDERE RONDES:\n{hist}\n\nBEWIJS (opgevraagde bestanden):\n{evidence or '(geen)'}\n\n"
            "Eindig met een JSON blok: {\"confidence_score\": 0-10, \"root_cause_key\": \"korte-sleutel\", "
            "\"evidence\": [], \"rules_out\": [], \"confirms\": [], \"file_requests\": [], \"next_test\": \"\"}")


def next_cr_id(log: str) -> str:
    nums = [int(m) for m in re.findall(r"^## CR-(\d+)", log, re.M)]
    return f"CR-{(max(nums) + 1) if nums else 1:03d}"


def append_error_log(root: str, symptoms: str, status: str, key: Optional[str], diags: List[Diagnosis]) -> str:
    path = os.path.join(root, ERROR_LOG)
    with file_lock(path):
        log = read_text(path) if os.path.exists(path) else "# Error Log — TheRoundtAIble code-red\n\n"
        cr = next_cr_id(log)
        lines = [f"## {cr} [{status}] — {symptoms[:80]}", "", f"**Date:** {iso_now()[:10]}",
                 f"**Root cause:** {key or 'unresolved'}", ""]
        for d in diags:
            lines.append(f"- {d.doctor} (ronde {d.round}): `{d.root_cause_key}` confidence {d.confidence_score}/10"
                         + (f"; next test: {d.next_test}" if d.next_test else ""))
        lines += ["", "---", "", ""]
        atomic_write_text(path, log + "\n".join(lines))
    return cr


def code_red_command(args, ui: UI) -> int:
    from .cli import is_writer, make_backends, spmd_cluster
    root = os.getcwd()
    config = load_config(root)
    cl = spmd_cluster(config)
    if cl is not None and cl.rank != 0:
        ui = UI(quiet=True)
    backends, _ = make_backends(config, ui, args)
    if not backends:
        raise ConfigError("No doctors available.")
    doctors = [k for k in sorted(config.knights, key=lambda k: k.priority) if k.adapter in backends]
    symptoms = args.symptoms
    ui.print(f"\n  CODE RED: {symptoms}\n", "bold", "red")
    transcript: List[str] = []
    latest: Dict[str, Diagnosis] = {}
    evidence = ""
    rounds = max(3, config.rules.max_rounds)
    key = None
    for rnd in range(1, rounds + 1):
        visible = list(transcript)
        pairs = [(backends[d.adapter], TurnRequest(f"codered:{d.name}", doctor_prompt(d.name, symptoms, rnd, visible,
                                                                                          evidence), rnd,
                                                   args.max_new_tokens)) for d in doctors]
        # blind round (and every round, here) runs the doctors concurrently: they see only rounds < rnd
        outs = pairs[0][0].execute_group(pairs, float(config.rules.timeout_per_turn_seconds)) \
            if len({b.group_key() for b, _ in pairs}) == 1 else [b.execute_many([r], 1e9)[0] for b, r in pairs]
        for d, out in zip(doctors, outs):
            if isinstance(out, BaseException):
                ui.error(f"  Dr. {d.name} is unavailable: {out}")
                continue
            transcript.append(f"### Dr. {d.name} ({PHASES.get(rnd, 'CONVERGENTIE')}, ronde {rnd}):\n{out.text}")
            dg = parse_diagnosis(out.text, d.name, rnd)
            ui.print(f"  Dr. {d.name}: " + (f"{dg.root_cause_key} ({dg.confidence_score}/10)" if dg else "(no verdict)"))
            if dg:
                latest[d.name] = dg
                if dg.file_requests:
                    ev = resolve_file_requests(dg.file_requests, root, config.rules.ignore)
                    evidence += ("\n\n" if evidence else "") + ev
        if rnd >= 2:
            key = check_convergence(latest)
            if key:
                break
    status = "OPEN" if key else "PARKED"
    if not is_writer():        # SPMD: rank 0 alone writes the project's error log
        return 0
    cr = append_error_log(root, symptoms, status, key, list(latest.values()))
    if key:
        ui.ok(f"\n  Diagnosis converged: {key} — logged as {cr} (OPEN until fixed).")
    else:
        ui.warn(f"\n  No convergence — parked as {cr}.")
    return 0
