"""Round engine: knights take turns until consensus, unanimous rejection or max rounds.

Parity: `src/orchestrator.ts:271-672` (``runDiscussion``), `:45-73` (runtime
fallback), `:114-139` (lead knight), `:145-157` (allowed scope), `:164-222` (file
requests; :mod:`.tools`), consensus/negative/escalation checks after every
*complete* round (`:539-649`).

Round modes (SURVEY §7.3 hard part 1):

``sequential`` (reference semantics). Knights speak one at a time; knight k in
round r sees rounds < r plus the round-r turns of earlier speakers; tool results
are visible to later speakers in the same round. Round 1 uses priority order, later
rounds (and every round of a continuation) a Fisher-Yates shuffle.

``parallel`` (MI355X mode). All knights of a round are launched concurrently and see
only rounds < r (like code-red's blind round, README.md:171). Knights hosted by the
same engine are decoded as one batch; engines on different GPUs run at the same
time. Entries are then recorded in speaking order, so ``discussion.md`` keeps the
reference shape.

Everything the reference does after a turn (parse, display, scope, tools, status,
chronicle) is unchanged. Additions: ``rounds.jsonl`` / ``metrics.jsonl`` per turn
(resume + observability), a session PID lock, and optional seeded shuffles.
"""
from __future__ import annotations

import random
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

from . import store
from .consensus import (check_consensus, check_negative_consensus, missing_scope_warning,
                        strip_consensus_json, summarize_consensus)
from .context import build_context
from .errors import AdapterError, classify_error
from .knights.base import KnightBackend, TurnRequest, TurnResult
from .prompt import (Prompt, Segment, TurnContext, build_turn_prompt_append, build_turn_prompt_reference,
                     build_turn_prompt_shared, transcript_entry_segments, KING_DEMAND)
from .tools import resolve_file_requests
from .types import (UNDEFINED, ConsensusBlock, ContinueOptions, KnightConfig, RoundEntry,
                    RoundtableConfig, SessionResult)
from .utils.clock import iso_now
from .utils.ui import NULL_UI, UI
from .verify import resolve_verify_commands

HINTS = {
    "not_installed": 'Is "{adapter}" configured with a model in adapter_config?',
    "timeout": "Consider increasing timeout_per_turn_seconds in config.",
    "auth": "Check your API key or subscription status.",
    "api": "The API returned an error. Try again later.",
    "oom": "Reduce max_new_tokens or context, or give the knight more GPUs.",
    "device": "The knight's GPU group was marked unhealthy.",
    "unknown": "",
}

THINKING = {
    "Claude": ["sharpens their arguments...", "is architecting a rebuttal...",
               "considers the elegant solution...", "mutters about clean code..."],
    "Gemini": ["drafts a 12-step plan...", "sees the bigger picture...", "is planning the plan...",
               "prepares a strategic response..."],
    "GPT": ["just wants to ship it...", "prepares a practical take...", "cuts through the noise...",
            "is getting impatient..."],
}

ROUND_HEADERS = [
    "KNIGHTS! DRAW YOUR KEYBOARDS!",
    "KNIGHTS! SPEAK NOW OR CODE SUFFERS! FOR KING AND KONG!",
    "EGOS CLASH, CODE SUFFERS!",
    "ONE LAST PLEA FOR SANITY!",
    "SPEAK NOW OR FOREVER HOLD YOUR MERGE CONFLICTS!",
]


def round_header(rnd: int) -> str:
    if 1 <= rnd <= len(ROUND_HEADERS):
        return f"ROUND {rnd} — {ROUND_HEADERS[rnd - 1]}"
    return f"ROUND {rnd} — FOR KING AND CODE!"


def select_lead_knight(knights: Sequence[KnightConfig], blocks: Sequence[ConsensusBlock]) -> KnightConfig:
    """Top scorer of the last round; ties -> lowest priority number (orchestrator.ts:114-139)."""
    if blocks:
        last = max(b.round for b in blocks)
        last_blocks = [b for b in blocks if b.round == last]
        if last_blocks:
            top = max(b.consensus_score for b in last_blocks)
            cands = [next((k for k in knights if k.name == b.knight), None)
                     for b in last_blocks if b.consensus_score == top]
            cands = sorted([k for k in cands if k is not None], key=lambda k: k.priority)
            if cands:
                return cands[0]
    return sorted(knights, key=lambda k: k.priority)[0]


def compute_allowed_files(blocks: Sequence[ConsensusBlock]) -> List[str]:
    seen: Dict[str, None] = {}
    for b in blocks:
        for f in b.files_to_modify or []:
            seen.setdefault(f, None)
    return list(seen)


@dataclass
class RunOptions:
    read_source: bool = False
    shuffle_seed: Optional[int] = None     # None = unseeded (reference Math.random semantics)
    round_mode: Optional[str] = None       # override config.rules.round_mode
    prompt_layout: Optional[str] = None    # override config.rules.prompt_layout
    max_new_tokens: Optional[int] = None   # per-turn cap passed to engine backends
    write_chronicle: bool = True
    # False: an SPMD mirror of a table another rank persists — the session/chronicle writes (and
    # their fsyncs) are dropped, reads still go to the project (bench.py / cli.py non-leader ranks)
    persist: bool = True


class _MirrorStore:
    """Store facade of a non-persisting orchestrator: reads pass through, writes are dropped."""
    _WRITES = frozenset({"append_round_entry", "append_metrics", "update_status", "write_discussion",
                         "write_decisions", "append_to_chronicle"})

    def __getattr__(self, name):
        if name == "create_session":
            return lambda root, topic: "<mirror>"
        if name in self._WRITES:
            return lambda *a, **k: None
        return getattr(store, name)


class Orchestrator:
    def __init__(self, config: RoundtableConfig, backends: Dict[str, KnightBackend], project_root: str,
                 ui: UI = NULL_UI, options: Optional[RunOptions] = None,
                 backend_factory: Optional[Callable[[str], Optional[KnightBackend]]] = None,
                 store_root: Optional[str] = None):
        self.config = config
        self.backends = backends
        self.root = project_root
        self.store_root = store_root or project_root   # where session/chronicle writes go (SPMD: rank 0 only)
        self.ui = ui
        self.opt = options or RunOptions()
        self.store = store if self.opt.persist else _MirrorStore()
        self.backend_factory = backend_factory
        self.rng = random.Random(self.opt.shuffle_seed)
        self.failures: List[Tuple[str, str, str]] = []   # (knight, error kind, message) per failed turn
        self.round_mode = self.opt.round_mode or config.rules.round_mode
        self.layout = self.opt.prompt_layout or config.rules.prompt_layout
        # append layout: transcript segments shared by every knight (grows append-only)
        self.transcript: List[Segment] = []
        self.table_id = ""   # prefix of engine sequence keys (unique per table when tables share engines)

    # ---- fallback (orchestrator.ts:45-73) ---------------------------------------------
    def _fallback_for(self, knight: KnightConfig) -> Optional[KnightBackend]:
        if not knight.fallback:
            return None
        key = f"__fallback_{knight.name}"
        fb = self.backends.get(key)
        if fb is None and self.backend_factory is not None:
            created = self.backend_factory(knight.fallback)
            if created is not None and created.is_available():
                self.backends[key] = created
                fb = created
        return fb

    # ---- prompt --------------------------------------------------------------------------
    def _prompt(self, knight: KnightConfig, ctx: TurnContext, visible: Sequence[RoundEntry], rnd: int,
                king_demand: bool, resolved_files: str, resolved_commands: str) -> Prompt:
        sem = self.config.rules.placeholder_semantics
        if self.layout == "append":
            return build_turn_prompt_append(knight, self.config.knights, ctx, self.transcript, rnd, semantics=sem)
        if self.layout == "shared":
            return build_turn_prompt_shared(knight, self.config.knights, ctx, self.transcript, rnd,
                                            shared_key=self.table_id + "@table", semantics=sem)
        return build_turn_prompt_reference(knight, self.config.knights, ctx, visible, king_demand=king_demand,
                                           resolved_files=resolved_files, resolved_commands=resolved_commands,
                                           semantics=sem)

    def _append_transcript(self, entry: RoundEntry, res: Optional[TurnResult]) -> None:
        if self.layout not in ("append", "shared"):
            return
        ids = res.ids if res is not None else None
        tok = res.tokenizer if res is not None else None
        self.transcript.extend(transcript_entry_segments(entry, ids, tok))

    # ---- one turn's bookkeeping (orchestrator.ts:444-520) -------------------------------
    def _record(self, knight: KnightConfig, backend: KnightBackend, rnd: int, res: TurnResult,
                all_rounds: List[RoundEntry], latest: Dict[str, ConsensusBlock],
                session_path: str, tool_state: Dict[str, str]) -> RoundEntry:
        consensus = backend.parse_consensus(res.text, rnd)
        entry = RoundEntry(knight=knight.name, round=rnd, response=res.text, consensus=consensus,
                           timestamp=iso_now(), metrics=dict(res.metrics))
        all_rounds.append(entry)
        self._append_transcript(entry, res)
        self.store.append_round_entry(session_path, entry)
        if res.metrics:
            self.store.append_metrics(session_path, {"knight": knight.name, "round": rnd, **res.metrics})
        ui = self.ui
        div = ui.knight(knight.name, "─" * 50)
        ui.print(div)
        ui.print(ui.knight(knight.name, f"  {knight.name}") + ui.paint(f" (Round {rnd})", "dim"))
        ui.print(div)
        shown = strip_consensus_json(res.text, "consensus_score").strip()
        ui.print("\n".join(f"  {l}" for l in shown.split("\n")), "white")
        if consensus is not None:
            latest[knight.name] = consensus
            s = consensus.consensus_score
            si = max(0, min(10, int(s))) if isinstance(s, (int, float)) else 0
            color = "green" if s >= 9 else "yellow" if s >= 6 else "red"
            ui.print("")
            ui.print(f"  {ui.knight(knight.name)} score: " + ui.paint(f"{'█' * si}{'░' * (10 - si)} {s}/10", color))
            if consensus.agrees_with:
                ui.dim(f"  Agrees with: {', '.join(map(str, consensus.agrees_with))}")
            if consensus.pending_issues:
                ui.warn(f"  Open issues: {', '.join(consensus.pending_issues)}")
            if consensus.file_requests:
                ui.dim(f"  Requesting files: {', '.join(map(str, consensus.file_requests))}")
                new = resolve_file_requests(consensus.file_requests, self.root, self.config.rules.ignore)
                if new:
                    tool_state["files"] += ("\n\n" if tool_state["files"] else "") + new
                    if self.layout in ("append", "shared"):
                        self.transcript.append(Segment(
                            f"\n\nOPGEVRAAGDE BESTANDEN (via file_requests van {knight.name}):\n{new}"))
            if consensus.verify_commands:
                ui.dim("  Verification commands:")
                new = resolve_verify_commands(consensus.verify_commands, self.root, log=ui.dim)
                if new:
                    tool_state["commands"] += ("\n\n" if tool_state["commands"] else "") + new
                    if self.layout in ("append", "shared"):
                        self.transcript.append(Segment(
                            f"\n\nVERIFICATIE RESULTATEN (via verify_commands van {knight.name}):\n{new}"))
        else:
            ui.warn("\n  (no consensus block found — the knight forgot the rules)")
        ui.print("")
        return entry

    def _report_failure(self, knight: KnightConfig, err: BaseException) -> None:
        c = classify_error(err, knight.name)
        self.failures.append((knight.name, c.kind, c.message))
        self.ui.error(f"  {knight.name} crashed and burned")
        self.ui.error(f"  Error ({c.kind}): {c.message}")
        hint = HINTS.get(c.kind, "").format(adapter=knight.adapter)
        if hint:
            self.ui.dim(f"  Hint: {hint}")

    def _execute_with_fallback(self, knight: KnightConfig, backend: KnightBackend,
                               req: TurnRequest, timeout_s: float) -> TurnResult:
        try:
            return _unwrap(backend.execute_many([req], timeout_s)[0])
        except Exception as primary:  # noqa: BLE001
            return self._execute_with_fallback_retry(knight, req, timeout_s, primary)

    # ---- main loop (steppable, so several tables can run in lockstep) -----------------------
    def begin(self, topic: str, continue_from: Optional[ContinueOptions] = None) -> None:
        cfg, rules, ui = self.config, self.config.rules, self.ui
        max_src = 200_000
        for k in cfg.knights:
            b = self.backends.get(k.adapter)
            if b is not None:
                m = b.max_source_chars()
                if m is not None and m < max_src:
                    max_src = m
        ctx = build_context(self.root, topic, rules.ignore, cfg.chronicle, self.opt.read_source, max_src,
                            warn=ui.warn)
        manifest = self.store.read_manifest(self.root)
        ctx.manifest_summary = self.store.manifest_summary(manifest)
        decrees = self.store.active_decrees(self.store.read_decree_log(self.root))
        ctx.decrees = self.store.format_decrees_for_prompt(decrees)
        if ctx.source_file_contents:
            ui.ok(f"  Context assembled (source: {round(len(ctx.source_file_contents) / 1024)}KB, "
                  f"manifest: {len(manifest['features'])} features, decrees: {len(decrees)})")
        else:
            ui.ok(f"  Context assembled (manifest: {len(manifest['features'])} features, decrees: {len(decrees)})")
        session_path = continue_from.session_path if continue_from else self.store.create_session(self.store_root, topic)
        if continue_from:
            ui.print("\n  The King has spoken. Back to the table, knights!\n", "bold", "yellow")
        else:
            ui.dim(f"  Session: {session_path}")
        self.topic = topic
        self.ctx = ctx
        self.cont = continue_from
        self.session_path = session_path
        self.ordered = sorted(cfg.knights, key=lambda k: k.priority)
        self.all_rounds: List[RoundEntry] = list(continue_from.all_rounds) if continue_from else []
        self.latest: Dict[str, ConsensusBlock] = {}
        self.tool_state = {"files": continue_from.resolved_files if continue_from else "",
                           "commands": continue_from.resolved_commands if continue_from else ""}
        if continue_from:
            for e in continue_from.all_rounds:
                if e.consensus:
                    self.latest[e.knight] = e.consensus
            if self.layout in ("append", "shared") and not self.transcript:
                for e in continue_from.all_rounds:
                    self.transcript.extend(transcript_entry_segments(e))
            if self.layout in ("append", "shared"):
                self.transcript.append(Segment("\n" + KING_DEMAND))
        self.start = continue_from.start_round if continue_from else 1
        self.end = self.start + rules.max_rounds - 1
        self.timeout_s = float(rules.timeout_per_turn_seconds)
        self.round_ms: List[float] = []
        self.result: Optional[SessionResult] = None

    def round_order(self, rnd: int) -> List[KnightConfig]:
        order = list(self.ordered)
        if not (rnd == self.start and not self.cont):
            self.rng.shuffle(order)
            self.ui.dim(f"  Speaking order: {' → '.join(k.name for k in order)}")
        self.ui.print(f"\n  {round_header(rnd)}\n", "bold", "blue")
        return order

    def plan_parallel(self, rnd: int, order: Sequence[KnightConfig]) -> List[Tuple[KnightConfig, KnightBackend, TurnRequest]]:
        """All turns of a parallel round: every knight sees only rounds < rnd."""
        visible = list(self.all_rounds)
        files, cmds = self.tool_state["files"], self.tool_state["commands"]
        plan = []
        predict = self._next_prompt_predictor(rnd, order)
        for knight in order:
            backend = self.backends.get(knight.adapter)
            if backend is None:
                self.ui.warn(f"  {knight.name} didn't show up today. Typical.")
                continue
            prompt = self._prompt(knight, self.ctx, visible, rnd, self.cont is not None, files, cmds)
            plan.append((knight, backend, TurnRequest(self.table_id + knight.name, prompt, rnd, self.opt.max_new_tokens,
                                                      speculate=predict)))
        self.store.update_status(self.session_path, phase="discussing", current_knight=None, round=rnd)
        return plan

    def _next_prompt_predictor(self, rnd: int, order: Sequence[KnightConfig]):
        """``shared`` layout: a function from the turns of this round finished so far (on one
        rank) to the table's round-``rnd + 1`` prompt as far as they determine it — the
        transcript plus this round's entries up to the first one not known yet, rendered exactly
        as :meth:`_record` will append them (entry header, reply ids, consensus annotation; an
        entry that triggers tool results ends the known part). A distributed pool prefills that
        shared prefix while the other ranks' replies are in flight (C1 overlap)."""
        if self.layout != "shared":
            return None
        transcript = list(self.transcript)

        def predict(done: Dict[str, TurnResult]) -> Optional[Prompt]:
            segs = list(transcript)
            n = 0
            for knight in order:
                res = done.get(self.table_id + knight.name)
                backend = self.backends.get(knight.adapter)
                if res is None or backend is None or isinstance(res, BaseException):
                    break
                consensus = backend.parse_consensus(res.text, rnd)
                entry = RoundEntry(knight=knight.name, round=rnd, response=res.text, consensus=consensus,
                                   timestamp="", metrics={})
                segs.extend(transcript_entry_segments(entry, res.ids, res.tokenizer))
                n += 1
                if consensus is not None and (consensus.file_requests or consensus.verify_commands):
                    break
            if n == 0:
                return None
            return build_turn_prompt_shared(order[0], self.config.knights, self.ctx, segs, rnd + 1,
                                            shared_key=self.table_id + "@table",
                                            semantics=self.config.rules.placeholder_semantics)
        return predict

    def record_parallel(self, rnd: int, order: Sequence[KnightConfig],
                        results: Dict[str, Union[TurnResult, BaseException]]) -> None:
        for knight in order:
            if self.table_id + knight.name not in results:
                continue
            out = results[self.table_id + knight.name]
            if isinstance(out, BaseException):
                self._report_failure(knight, out)
                continue
            self._record(knight, self.backends[knight.adapter], rnd, out, self.all_rounds, self.latest,
                         self.session_path, self.tool_state)

    def plan_turn(self, rnd: int, knight: KnightConfig) -> Optional[Tuple[KnightConfig, KnightBackend, TurnRequest]]:
        """One sequential-mode turn: the prompt sees every entry recorded so far (orchestrator.ts:397-425)."""
        backend = self.backends.get(knight.adapter)
        if backend is None:
            self.ui.warn(f"  {knight.name} didn't show up today. Typical.")
            return None
        self.store.update_status(self.session_path, phase="discussing", current_knight=knight.name, round=rnd)
        prompt = self._prompt(knight, self.ctx, self.all_rounds, rnd, self.cont is not None,
                              self.tool_state["files"], self.tool_state["commands"])
        msgs = THINKING.get(knight.name, ["is thinking...", "prepares their response..."])
        self.ui.print(f"  {knight.name} {msgs[self.rng.randrange(len(msgs))]}", "dim")
        return knight, backend, TurnRequest(self.table_id + knight.name, prompt, rnd, self.opt.max_new_tokens)

    def record_turn(self, rnd: int, knight: KnightConfig, backend: KnightBackend,
                    res: Union[TurnResult, BaseException]) -> None:
        if isinstance(res, BaseException):
            self._report_failure(knight, res)   # skip the knight, continue the round
            return
        self._record(knight, backend, rnd, res, self.all_rounds, self.latest, self.session_path, self.tool_state)

    def run_sequential_round(self, rnd: int, order: Sequence[KnightConfig]) -> None:
        for knight in order:
            planned = self.plan_turn(rnd, knight)
            if planned is None:
                continue
            _, backend, req = planned
            try:
                res = self._execute_with_fallback(knight, backend, req, self.timeout_s)
            except Exception as e:  # noqa: BLE001 - skip the knight, continue the round
                res = e
            self.record_turn(rnd, knight, backend, res)

    def execute_plan(self, plan) -> Dict[str, Union[TurnResult, BaseException]]:
        """Run planned turns grouped by backend group (one batched decode per engine), groups concurrently."""
        groups: Dict[object, List[Tuple[KnightConfig, KnightBackend, TurnRequest]]] = {}
        for item in plan:
            groups.setdefault(item[1].group_key(), []).append(item)
        results: Dict[str, Union[TurnResult, BaseException]] = {}

        def run_group(members):
            outs = members[0][1].execute_group([(b, r) for _, b, r in members], self.timeout_s)
            return [(k, r, o) for (k, _, r), o in zip(members, outs)]

        with ThreadPoolExecutor(max_workers=max(1, len(groups))) as ex:
            for triples in ex.map(run_group, list(groups.values())):
                for knight, req, out in triples:
                    if isinstance(out, BaseException):
                        try:
                            out = self._execute_with_fallback_retry(knight, req, self.timeout_s, out)
                        except Exception as e:  # noqa: BLE001
                            out = e
                    results[req.seq_key] = out
        return results

    def end_round(self, rnd: int, round_ms: float) -> Optional[SessionResult]:
        """Persist + consensus / rejection / escalation checks after a complete round (orchestrator.ts:539-649)."""
        cfg, rules, ui = self.config, self.config.rules, self.ui
        topic, session_path, all_rounds, latest = self.topic, self.session_path, self.all_rounds, self.latest
        self.round_ms.append(round_ms)
        self.store.append_metrics(session_path, {"round": rnd, "round_ms": round_ms, "mode": self.round_mode,
                                            "layout": self.layout})
        self.store.write_discussion(session_path, all_rounds)
        current = list(latest.values())
        tool_state = self.tool_state
        if check_consensus(current, rules.consensus_threshold):
            ui.print("\n  Against all odds... they actually agree.", "bold", "green")
            ui.print(summarize_consensus(current))
            for b in current:
                w = missing_scope_warning(b)
                if w:
                    ui.warn(w)
            allowed = compute_allowed_files(current)
            if allowed:
                ui.print(f"\n  Scope: {len(allowed)} file(s) in modification scope:", "cyan")
                for f in allowed:
                    is_new = f.upper().startswith("NEW:")
                    ui.print(f"    + {f[4:]} (new)" if is_new else f"    ~ {f}", "green" if is_new else "dim")
            proposal = next((e.consensus.proposal for e in reversed(all_rounds)
                             if e.consensus is not None and _truthy(e.consensus.proposal)), None)
            if proposal is None:
                proposal = all_rounds[-1].response if all_rounds else "No proposal text available."
            proposal = proposal if isinstance(proposal, str) else _js_string(proposal)
            lead = select_lead_knight(cfg.knights, current)
            self.store.write_decisions(session_path, topic, proposal, all_rounds)
            self.store.update_status(session_path, phase="consensus_reached", consensus_reached=True, round=rnd,
                                allowed_files=allowed if allowed else UNDEFINED, lead_knight=lead.name)
            if self.opt.write_chronicle:
                self.store.append_to_chronicle(self.store_root, cfg.chronicle, topic=topic,
                                          outcome=f"Consensus in {rnd} round(s). Lead Knight: {lead.name}.\n\n{proposal}",
                                          knights=[b.knight for b in current], date=iso_now()[:10])
            self.result = SessionResult(session_path, True, rnd, proposal, current, all_rounds,
                                        resolved_files=tool_state["files"], resolved_commands=tool_state["commands"],
                                        lead_knight=lead.name)
            return self.result
        if check_negative_consensus(current):
            ui.print("\n  A rare sight — the knights actually agree on something.", "bold", "red")
            ui.print("  Unfortunately, they agree that your idea is terrible.\n", "bold", "red")
            ui.print(summarize_consensus(current))
            rejection = "\n\n---\n\n".join(f"## {e.knight}\n\n{e.response}" for e in all_rounds if e.round == rnd)
            self.store.write_decisions(session_path, topic, rejection, all_rounds)
            self.store.update_status(session_path, phase="consensus_reached", consensus_reached=True, round=rnd)
            if self.opt.write_chronicle:
                self.store.append_to_chronicle(self.store_root, cfg.chronicle, topic=topic,
                                          outcome=f"Unanimous rejection in {rnd} round(s). All knights advise against this.",
                                          knights=[b.knight for b in current], date=iso_now()[:10])
            self.result = SessionResult(session_path, True, rnd, rejection, current, all_rounds,
                                        unanimous_rejection=True, resolved_files=tool_state["files"],
                                        resolved_commands=tool_state["commands"])
            return self.result
        if rnd >= rules.escalate_to_user_after and rnd < self.end:
            ui.warn(f"\n  Round {rnd}: Still no consensus. {self.end - rnd} round(s) left before escalation.")
        return None

    def finish(self) -> SessionResult:
        if self.result is not None:
            return self.result
        self.ui.print("\n  The knights have agreed to disagree. Your move.", "bold", "yellow")
        self.ui.print(summarize_consensus(list(self.latest.values())))
        self.store.update_status(self.session_path, phase="escalated", consensus_reached=False, round=self.end)
        self.result = SessionResult(self.session_path, False, self.end, None, list(self.latest.values()),
                                    self.all_rounds, resolved_files=self.tool_state["files"],
                                    resolved_commands=self.tool_state["commands"])
        return self.result

    def run(self, topic: str, continue_from: Optional[ContinueOptions] = None) -> SessionResult:
        self.begin(topic, continue_from)
        for rnd in range(self.start, self.end + 1):
            order = self.round_order(rnd)
            t0 = time.perf_counter()
            if self.round_mode == "parallel":
                plan = self.plan_parallel(rnd, order)
                self.record_parallel(rnd, order, self.execute_plan(plan))
            else:
                self.run_sequential_round(rnd, order)
            done = self.end_round(rnd, (time.perf_counter() - t0) * 1e3)
            if done is not None:
                return done
        return self.finish()

    def _execute_with_fallback_retry(self, knight, req, timeout_s, err):
        fb = self._fallback_for(knight)
        if fb is None:
            raise err
        self.ui.warn(f"  {knight.name} primary adapter failed, switching to fallback ({knight.fallback})...")
        return _unwrap(fb.execute_many([req], timeout_s)[0])


def run_tables_parallel(tables: Sequence[Orchestrator], topics: Sequence[str],
                        on_round: Optional[Callable[[int, float], None]] = None) -> List[SessionResult]:
    """Run several independent tables in lockstep (parallel round mode): each round, every
    still-open table plans its turns, all turns execute as ONE batch (grouped per engine /
    distributed pool), then each table records and checks consensus on its own."""
    for i, (t, topic) in enumerate(zip(tables, topics)):
        if len(tables) > 1 and not t.table_id:
            t.table_id = f"t{i}/"
        t.begin(topic)
    open_ = list(tables)
    rnd = min(t.start for t in tables)
    while open_:
        t0 = time.perf_counter()
        orders = {id(t): t.round_order(rnd) for t in open_}
        plans = {id(t): t.plan_parallel(rnd, orders[id(t)]) for t in open_}
        merged = [item for t in open_ for item in plans[id(t)]]
        results = open_[0].execute_plan(merged)
        for t in open_:
            t.record_parallel(rnd, orders[id(t)], results)
        ms = (time.perf_counter() - t0) * 1e3
        still = []
        for t in open_:
            if t.end_round(rnd, ms) is None and rnd < t.end:
                still.append(t)
            elif t.result is None:
                t.finish()
        open_ = still
        if on_round is not None:
            on_round(rnd, ms)
        rnd += 1
    return [t.finish() for t in tables]


def run_tables_sequential(tables: Sequence[Orchestrator], topics: Sequence[str],
                          on_round: Optional[Callable[[int, float], None]] = None) -> List[SessionResult]:
    """Several independent tables in reference (sequential) round mode, in lockstep by
    speaking slot: the k-th speaker of every open table runs in one batch, each seeing its
    own table's earlier speakers of the round (orchestrator.ts:361-536 visibility)."""
    for i, (t, topic) in enumerate(zip(tables, topics)):
        if len(tables) > 1 and not t.table_id:
            t.table_id = f"t{i}/"
        t.begin(topic)
    open_ = list(tables)
    rnd = min(t.start for t in tables)
    while open_:
        t0 = time.perf_counter()
        orders = {id(t): t.round_order(rnd) for t in open_}
        for k in range(max(len(o) for o in orders.values())):
            planned = []
            for t in open_:
                if k < len(orders[id(t)]):
                    item = t.plan_turn(rnd, orders[id(t)][k])
                    if item is not None:
                        planned.append((t, item))
            if not planned:
                continue
            results = open_[0].execute_plan([item for _, item in planned])
            for t, (knight, backend, req) in planned:
                t.record_turn(rnd, knight, backend, results[req.seq_key])
        ms = (time.perf_counter() - t0) * 1e3
        still = []
        for t in open_:
            if t.end_round(rnd, ms) is None and rnd < t.end:
                still.append(t)
            elif t.result is None:
                t.finish()
        open_ = still
        if on_round is not None:
            on_round(rnd, ms)
        rnd += 1
    return [t.finish() for t in tables]


def _unwrap(x):
    if isinstance(x, BaseException):
        raise x
    return x


def _truthy(v) -> bool:
    return v not in (None, "", 0, False)


def _js_string(v) -> str:
    import json
    if isinstance(v, (dict, list)):
        return json.dumps(v, ensure_ascii=False)
    return str(v)
