"""``roundtable`` CLI (reference `src/index.ts:48-182` + `src/commands/*.ts`).

Commands: init, discuss, summon, apply, status, list, chronicle, decrees,
manifest {list,add,deprecate,check}, code-red, bench. ``main`` is the single error
sink: every command raises, ``main`` formats and returns the exit code (index.ts:25-46).
Interactive questions read stdin; every one also has a flag so scripts and CI can
run non-interactively (EOF on stdin = the default answer).
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import List, Optional

from . import __version__, store
from .config import DEFAULT_CAPABILITIES, generate_config, load_config, write_config
from .errors import ConfigError, RoundtableError, format_error, get_exit_code
from .types import ContinueOptions
from .utils.ui import UI


# ---- prompts ------------------------------------------------------------------------------------
_CLUSTER = None   # set when discuss/summon run under torchrun (one process per GPU, SPMD)


def spmd_cluster(config=None):
    """The torchrun cluster for SPMD commands (None for a single-process run). A config whose
    engine knights all run on the CPU gets gloo ranks (tests / CPU plumbing)."""
    global _CLUSTER
    if _CLUSTER is None and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from .parallel.cluster import init_cluster
        cpu = False
        timeout = 1800
        if config is not None:
            from .parallel.launch import collective_timeout_s, ranks_needed
            cpu = ranks_needed(config)[2]
            timeout = collective_timeout_s(config)
        _CLUSTER = init_cluster(prefer_gpu=not cpu, timeout_s=timeout)
        _start_guard(_CLUSTER, config)
    return _CLUSTER


def _start_guard(cl, config) -> None:
    """Containment for SPMD commands (utils/failsafe.py, as in bench.py): engine loading, K9
    set-up, graph capture and every turn batch run under time limits on every rank; a rank that
    raises or stalls past its limit ends the whole command with one message naming the stage and
    rank (exit code 2), instead of its peers waiting in a collective. Turn batches carry their own
    limit (knights/distributed.py: the turn timeout per knight group, plus margin)."""
    if cl is None or not cl.distributed:
        return
    from .utils import failsafe
    t = float(getattr(getattr(config, "rules", None), "timeout_per_turn_seconds", 120) or 120)

    def report(rec: dict) -> None:
        sys.stderr.write(failsafe.describe(rec, "roundtable") + "\n")

    failsafe.RunGuard(cl.rank, cl.world, report, default_s=float("inf"), exit_code=2,
                      limits={"engine_load": 900.0, "k9_create": 900.0, "capture": t + 120.0}).start()


def make_backends(config, ui: UI, args, only_knight: Optional[str] = None):
    """(backends, factory) for a command. Under torchrun (SPMD, parallel/launch.py self-launch):
    every rank builds the engines placed on it and one RemoteKnight per adapter id
    (knights/spmd.py); otherwise in-process engines (one per GPU / model). ``only_knight``: build
    just that knight's backend (apply's lead knight)."""
    cl = spmd_cluster(config)
    if cl is not None and cl.distributed:
        import copy
        from .knights.spmd import build_spmd_backends
        cfg = config
        if only_knight is not None:
            cfg = copy.copy(config)
            cfg.knights = [k for k in config.knights if k.name == only_knight] or config.knights[:1]
        backends, _pool = build_spmd_backends(cfg, cl, ui, getattr(args, "max_new_tokens", None))
        return backends, None
    if only_knight is not None:
        from .knights.registry import BackendFactory
        k = next((k for k in config.knights if k.name == only_knight), config.knights[0])
        b = BackendFactory(config, device_override=getattr(args, "device", None)).create(k.adapter)
        return ({k.adapter: b} if b is not None else {}), None
    return _make_backends(config, ui, getattr(args, "device", None))


def is_writer() -> bool:
    """Only rank 0 writes project files / asks the King in an SPMD run."""
    return _CLUSTER is None or _CLUSTER.rank == 0


def ask(ui: UI, question: str, default: str = "") -> str:
    line = None
    if is_writer():
        ui.print(question)
        try:
            line = sys.stdin.readline()
        except (EOFError, OSError):
            line = None
    if _CLUSTER is not None and _CLUSTER.distributed:
        # every rank takes the King's answer (a person: no containment timeout on this wait)
        line = _CLUSTER.broadcast_object(line, src=0, wait=True)
    if not line:
        return default
    return line.strip() or default


def confirm(ui: UI, question: str, default_yes: bool = True) -> bool:
    hint = "[Y/n]" if default_yes else "[y/N]"
    ans = ask(ui, f"{question} {hint}", "y" if default_yes else "n").lower()
    return ans in ("y", "yes", "ja")


# ---- init ---------------------------------------------------------------------------------------
def gpu_inventory():
    """GPU inventory (name, HBM, CUs, xGMI links) scouted in a child process, so this process
    never initializes HIP (parallel/placement.py). ``ROUNDTABLE_FAKE_GPUS`` (a JSON inventory)
    replaces the probe in tests."""
    from .parallel.placement import Inventory, scout_gpus
    fake = os.environ.get("ROUNDTABLE_FAKE_GPUS")
    if fake:
        import json as _json
        return Inventory.from_json(_json.loads(fake))
    return scout_gpus()


CLI_TOOLS = {"claude-cli": "claude", "gemini-cli": "gemini", "openai-cli": "codex"}
API_FALLBACKS = (("claude-api", "ANTHROPIC_API_KEY", "Anthropic"), ("gemini-api", "GEMINI_API_KEY", "Gemini"),
                 ("openai-api", "OPENAI_API_KEY", "OpenAI"))


def detect_tools(commands=("claude", "gemini", "codex")) -> dict:
    """``<cmd> --version`` for every vendor CLI, in parallel (init.ts:96-113)."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor

    def probe(cmd):
        try:
            return subprocess.run([cmd, "--version"], capture_output=True, timeout=10).returncode == 0
        except (OSError, subprocess.SubprocessError):
            return False
    with ThreadPoolExecutor(max_workers=len(commands)) as ex:
        return dict(zip(commands, ex.map(probe, commands)))


def ask_secret(ui: UI, question: str) -> str:
    """Masked input (init.ts:49-91 raw-mode reader); empty when stdin is not a terminal."""
    import getpass
    if not sys.stdin.isatty():
        return ""
    try:
        return getpass.getpass(question + " ").strip()
    except (EOFError, KeyboardInterrupt):
        return ""


def _ask_fallback_key(ui: UI, knights, external) -> None:
    from .store.keys import save_key
    for i, (aid, var, label) in enumerate(API_FALLBACKS, start=1):
        ui.print(f"    {i}. {label} ({aid})")
    raw = ask(ui, f"  Which provider? [1-{len(API_FALLBACKS)}]", "")
    if not raw.isdigit() or not 1 <= int(raw) <= len(API_FALLBACKS):
        return
    aid, var, label = API_FALLBACKS[int(raw) - 1]
    key = ask_secret(ui, f"  {label} API key:")
    if not key:
        ui.dim("  No key entered; no fallback added.")
        return
    save_key(var, key)
    names = ", ".join(k["name"] for k in knights)
    who = ask(ui, f"  Fallback for which knight? ({names})", knights[0]["name"])
    for k in knights:
        if k["name"].lower() == who.lower():
            k["fallback"] = aid
            external[aid] = {"backend": "external"}
            ui.ok(f"  {k['name']} falls back to {aid}; key saved to ~/.theroundtaible/keys.json")
            return


def cmd_init(args, ui: UI) -> int:
    root = os.getcwd()
    rt = os.path.join(root, ".roundtable")
    if os.path.exists(rt) and not args.yes:
        ui.warn("\n  The roundtable already exists in this project.")
        if not confirm(ui, "  Reinitialize? This will overwrite your config.", False):
            ui.dim("  Wise choice. The table stands.")
            return 0
    ui.print("\n  Welcome to TheRoundtAIble (MI355X engine)\n", "bold")
    ui.dim(f"  Version: v{__version__}")
    project = args.project or (os.path.basename(root) if args.yes else ask(ui, f"  Project name? ({os.path.basename(root)})", os.path.basename(root)))
    language = args.language or ("nl" if args.yes else ask(ui, "  Discussion language? (nl)", "nl"))
    inv = gpu_inventory()
    gpus = inv.gpus
    if gpus:
        g = gpus[0]
        xgmi = sum(1 for v in inv.links.values() if v == "XGMI")
        ui.ok(f"  Scouting complete: {len(gpus)} x {g.name or 'GPU'} ({g.arch}), "
              f"{g.hbm_bytes / (1 << 30):.0f} GiB HBM each, {g.cus} CUs"
              + (f", {xgmi} xGMI link(s)" if inv.links else ""))
    else:
        ui.ok("  Scouting complete: 0 GPU(s) visible — knights will run on CPU")
    seats = [("Claude", "claude-cli"), ("Gemini", "gemini-cli"), ("GPT", "openai-cli")][:max(1, min(3, args.knights))]
    extra = max(0, args.knights - 3)
    knights = []
    adapter_engine = {}
    for i, (name, adapter) in enumerate(seats):
        if args.yes or confirm(ui, f"  Seat {name} at the table?", True):
            knights.append({"name": name, "adapter": adapter})
    for j in range(extra):
        knights.append({"name": f"Knight{j + 4}", "adapter": f"local-llm-knight{j + 4}",
                        "capabilities": ["code", "logic"]})
    # local checkpoints (init.ts:361-373 seats detected local models as local-llm-<slug> knights)
    from .utils.local_detect import detect_local_models
    local_engine = {}
    found = detect_local_models(project_root=root)
    if found:
        ui.ok(f"  Found {len(found)} local checkpoint(s): " + ", ".join(m.name for m in found))
    for m in found:
        if m.preset is None:
            continue
        if args.local_models or (not args.yes and confirm(ui, f"  Seat {m.name} ({m.preset}) at the table?", False)):
            adapter = f"local-llm-{m.adapter_slug()}"
            knights.append({"name": m.name, "adapter": adapter, "capabilities": ["code", "logic"]})
            local_engine[adapter] = {"model": m.preset, "weights": m.path, "model_overrides": m.overrides}
    # running LM Studio / Ollama servers (init.ts:255,361-373): external local-llm seats over HTTP
    external = {}
    if args.servers:
        from .utils.local_detect import detect_local_servers
        for sm in detect_local_servers():
            adapter = f"local-llm-{sm.adapter_slug()}"
            if any(k["adapter"] == adapter for k in knights):
                continue
            knights.append({"name": sm.name, "adapter": adapter, "capabilities": ["code", "logic"]})
            external[adapter] = sm.adapter_config()
            ui.ok(f"  Found {sm.name} on {sm.source} ({sm.endpoint})")
    # installed vendor CLIs (init.ts:96-113): seat them on their own transport instead of the engine
    if args.external_clis:
        tools = detect_tools()
        for k in knights:
            if k["adapter"] in CLI_TOOLS and tools.get(CLI_TOOLS[k["adapter"]]):
                external[k["adapter"]] = {"backend": "external"}
                ui.ok(f"  {k['name']}: {CLI_TOOLS[k['adapter']]} CLI found, seated on its own transport")
    # API-key fallback (init.ts:306-323): masked input, stored in ~/.theroundtaible/keys.json
    if not args.yes and knights and confirm(ui, "  Add an API key as fallback for a knight?", False):
        _ask_fallback_key(ui, knights, external)
    if not knights:
        ui.error("\n  A roundtable with no knights is just a table.")
        return 0
    placement = None
    if args.tp is not None or not gpus:
        tp = args.tp or 1      # manual: knights dealt round-robin, tp consecutive GPUs each
        for i, k in enumerate(knights):
            eng = dict(local_engine.get(k["adapter"], {"model": args.model}), tp=tp)
            if gpus:
                g0 = (i * tp) % len(gpus)
                eng["gpus"] = [(g0 + t) % len(gpus) for t in range(tp)]
            else:
                eng["device"] = "cpu"
            adapter_engine[k["adapter"]] = eng
    else:
        # automatic placement: tp by memory fit + decode-step target, same-model knights together
        from .parallel.placement import plan_placement
        seats = [{"name": k["adapter"], **local_engine.get(k["adapter"], {"model": args.model})} for k in knights]
        from .parallel.placement import PlacementPolicy
        plans = plan_placement([{"name": s_["name"], "model": s_["model"], "overrides": s_.get("model_overrides")}
                                for s_ in seats], inv,
                               PlacementPolicy(mode=getattr(args, "placement", None) or "auto"))
        for pl in plans:
            for aid in pl.knights:
                adapter_engine[aid] = dict(local_engine.get(aid, {"model": args.model}), tp=pl.tp, gpus=pl.gpus)
            ui.ok(f"  Placement: {pl.model} x{len(pl.knights)} -> GPU {','.join(map(str, pl.gpus))} "
                  f"(tp={pl.tp}, {pl.weight_gib_per_gpu} GiB weights/GPU, ~{pl.step_ms} ms/step: {pl.reason})")
        placement = {"inventory": inv.to_json(),
                     "groups": [{"model": pl.model, "tp": pl.tp, "gpus": pl.gpus, "adapters": pl.knights,
                                 "reason": pl.reason, "round_ms": pl.round_ms} for pl in plans]}
    eng_top = {"default_model": args.model, "weights": args.weights, "dtype": "bf16",
               "max_new_tokens": args.max_new_tokens}
    if placement is not None:
        eng_top["placement"] = placement
    cfg = generate_config(project, language, knights, engine=eng_top, adapter_engine=adapter_engine)
    for aid, ac in external.items():
        cfg["adapter_config"].setdefault(aid, {}).update(ac)
        if aid in adapter_engine and "endpoint" in ac:
            cfg["adapter_config"][aid].pop("engine", None)
    for k in knights:
        if k["adapter"].startswith("local-llm") and k["adapter"] not in external:
            model = adapter_engine[k["adapter"]]["model"]
            cfg["adapter_config"][k["adapter"]].update({"endpoint": "engine://local", "model": model,
                                                        "name": k["name"]})
    os.makedirs(os.path.join(rt, "sessions"), exist_ok=True)
    write_config(root, cfg)
    from .utils.atomic import atomic_write_text
    from .store.chronicle import INIT_HEADER
    from .types import dumps_js
    from .utils.clock import iso_now
    atomic_write_text(os.path.join(rt, "chronicle.md"), INIT_HEADER)
    atomic_write_text(os.path.join(rt, "manifest.json"),
                      dumps_js({"version": "1.0", "last_updated": iso_now(), "features": []}))
    ui.ok("\n  TheRoundtAIble is ready.\n")
    ui.print(f"    Project:   {project}")
    ui.print(f"    Language:  {language}")
    ui.print(f"    Knights:   {', '.join(k['name'] for k in knights)} ({args.model})")
    from .config import load_config as _load
    from .parallel.launch import ranks_needed
    n, why, _cpu = ranks_needed(_load(root))
    if n > 1:
        ui.dim(f"\n  Placement needs {n} GPU ranks ({why}): `roundtable discuss` launches them itself "
               f"(one process per GPU, torch.distributed over RCCL).")
    ui.dim('\n  The table is set. Run `roundtable discuss "your question"` to begin.\n')
    return 0


# ---- discuss / summon ---------------------------------------------------------------------------
def _make_backends(config, ui: UI, device: Optional[str] = None):
    from .knights.registry import BackendFactory, initialize_backends
    factory = BackendFactory(config, device_override=device)
    return initialize_backends(config, ui, factory), factory


def js_parse_int(text: str) -> Optional[int]:
    """JavaScript ``parseInt(text)`` (no radix, discuss.ts:181): leading whitespace and a sign,
    a ``0x`` prefix means hex, then the longest digit run — ``"2 "`` and ``"2abc"`` are 2;
    ``None`` where JS gives NaN."""
    import re
    t = (text or "").lstrip()
    if re.match(r"[+-]?0[xX]", t) and not re.match(r"[+-]?0[xX][0-9a-fA-F]", t):
        return None                       # "0x" with no hex digit: NaN
    m = re.match(r"([+-]?)(0[xX][0-9a-fA-F]+|\d+)", t)
    if m is None:
        return None
    body = m.group(2)
    v = int(body[2:], 16) if body[:2] in ("0x", "0X") else int(body)
    return -v if m.group(1) == "-" else v


def last_proposals(all_rounds):
    """(discuss.ts:229-260) last entry per knight with a one-line summary."""
    import re
    last = {}
    for e in all_rounds:
        last[e.knight] = e
    out = []
    for e in last.values():
        score = e.consensus.consensus_score if e.consensus else 0
        cleaned = re.sub(r"```json[\s\S]*?```", "", e.response)
        cleaned = re.sub(r'\{[^{}]*"consensus_score"[^{}]*\}', "", cleaned).strip()
        lines = [l for l in cleaned.split("\n") if len(l.strip()) > 10]
        summary = lines[0].strip() if lines else "No summary available"
        if len(summary) > 80:
            summary = summary[:77] + "..."
        out.append({"knight": e.knight, "score": score, "summary": summary, "full": e.response})
    return out


def discuss(topic: str, args, ui: UI) -> int:
    from .orchestrator import Orchestrator, RunOptions
    root = os.getcwd()
    config = load_config(root)
    cl = spmd_cluster(config)
    if cl is not None and cl.rank != 0:
        ui = UI(quiet=True)
    ui.print(f'\n  Topic: "{topic}"\n', "bold")
    ui.dim("  Summoning the knights to the table...\n")
    store_root = root
    if cl is not None and cl.distributed:
        # SPMD: every rank runs this program; knights run where they are placed (knights/spmd.py)
        import tempfile
        backends, factory = make_backends(config, ui, args)
        if cl.rank != 0:
            store_root = tempfile.mkdtemp(prefix=f"roundtable-rank{cl.rank}-")   # mirror writes, discarded
        if args.seed is None:   # one speaking order for all ranks
            import random
            args.seed = cl.broadcast_object(random.SystemRandom().randrange(1 << 31) if cl.rank == 0 else None)
    else:
        backends, factory = _make_backends(config, ui, getattr(args, "device", None))
    if not backends:
        raise ConfigError("A roundtable with no knights is just a table.",
                          hint="Configure at least one knight adapter with an engine model.")
    names = [next((k.name for k in config.knights if k.adapter == a), a) for a in backends]
    ui.dim(f"  {', '.join(names)} {'takes' if len(names) == 1 else 'take'} their seat{'' if len(names) == 1 else 's'}.\n")
    if args.read_codebase is None:
        ans = ask(ui, "  Shall the knights read the codebase first? Read codebase? [Y/N]", "n").lower()
        read_src = ans in ("y", "yes")
    else:
        read_src = args.read_codebase
    opts = RunOptions(read_source=read_src, shuffle_seed=args.seed, round_mode=args.round_mode,
                      prompt_layout=args.layout, max_new_tokens=args.max_new_tokens)
    orch = Orchestrator(config, backends, root, ui, opts, backend_factory=factory, store_root=store_root)
    cont = None
    if args.resume:
        cont = _resume_state(root, args.resume)
    result = orch.run(topic, cont)
    while True:
        ui.print("\n" + "=" * 50, "bold")
        if result.consensus:
            if result.unanimous_rejection:
                ui.print("  The knights unanimously reject this proposal.", "bold", "red")
                ui.dim(f"  Rounds: {result.rounds}\n  Session: {result.session_path}")
            else:
                ui.print("  A miracle has occurred. The knights actually agree.", "bold", "green")
                ui.dim(f"  Rounds: {result.rounds}\n  Session: {result.session_path}")
                ui.dim(f"  Read the decision: {result.session_path}/decisions.md\n")
                _kings_decree(root, topic, result, args, ui)
            break
        action = _no_consensus(root, topic, result, args, ui)
        if action != "send_back":
            break
        ui.print("=" * 50, "bold")
        cont = ContinueOptions(result.session_path, result.all_rounds, result.rounds + 1,
                               result.resolved_files, result.resolved_commands)
        args.choice = None  # a scripted choice applies once
        result = orch.run(topic, cont)
    ui.print("=" * 50 + "\n", "bold")
    return 0


def _resume_state(root: str, session: str) -> ContinueOptions:
    """``--resume <session>``: continue a crashed/escalated discussion from rounds.jsonl."""
    from .errors import SessionError
    path = session if os.path.isabs(session) else os.path.join(root, ".roundtable", "sessions", session)
    if session == "latest":
        info = store.find_latest_session(root)
        if info is None:
            raise SessionError("No session to resume.")
        path = info.path
    if not os.path.isdir(path):
        raise SessionError(f"Session not found: {session}")
    entries = store.load_round_entries(path)
    last = max((e.round for e in entries), default=0)
    return ContinueOptions(path, entries, last + 1)


def _kings_decree(root, topic, result, args, ui: UI) -> None:
    """Decree after consensus (decree.ts:11-23 + TODO.md:95-100): self / later / reject."""
    choice = args.decree
    if choice is None:
        return
    name = os.path.basename(result.session_path)
    if choice == "later":
        if is_writer():
            e = store.add_decree_entry(root, "deferred", name, topic, args.decree_reason)
            ui.dim(f"  Decree {e['id']}: deferred.")
    elif choice == "reject":
        if is_writer():
            e = store.add_decree_entry(root, "rejected_no_apply", name, topic, args.decree_reason)
            ui.dim(f"  Decree {e['id']}: rejected, no apply.")


def _no_consensus(root, topic, result, args, ui: UI) -> str:
    ui.print("  The knights have agreed to disagree. As usual.", "bold", "yellow")
    ui.dim(f"  Rounds: {result.rounds}\n  Session: {result.session_path}")
    props = last_proposals(result.all_rounds)
    if not props:
        ui.dim("\n  No proposals to choose from. The knights were useless today.")
        return "done"
    ui.print("\n  But YOU are the King. The final word is yours.\n", "bold")
    for i, p in enumerate(props, start=1):
        ui.print(f"  {i}. {p['knight']} ({p['score']}/10) — {p['summary']}")
    ui.print(f"  {len(props) + 1}. Send them back — they must reach unanimity!")
    raw = str(args.choice) if args.choice is not None else ask(ui, f"  What say you, Your Majesty? [1-{len(props) + 1}]", "")
    choice = js_parse_int(raw)
    if choice is None or choice < 1 or choice > len(props) + 1:
        ui.dim("  The King waves dismissively. Perhaps another time.")
        return "done"
    if choice == len(props) + 1:
        return "send_back"
    chosen = props[choice - 1]
    ui.print(f"\n  The King has chosen {chosen['knight']}'s advice. So it shall be.", "bold")
    store.write_decisions(result.session_path, topic, chosen["full"], result.all_rounds)
    store.update_status(result.session_path, phase="consensus_reached", consensus_reached=True,
                        lead_knight=chosen["knight"])
    ui.dim(f"  Read the decision: {result.session_path}/decisions.md\n")
    return "done"


def cmd_discuss(args, ui: UI) -> int:
    return discuss(args.topic, args, ui)


def cmd_summon(args, ui: UI) -> int:
    from .gitutil import git_branch, git_diff, recent_commits
    root = os.getcwd()
    load_config(root)
    ui.dim("\n  Reading the git scrolls...\n")
    diff, branch, commits = git_diff(root), git_branch(root), recent_commits(3, root)
    if not diff:
        ui.warn("  Nothing to review. The code rests in peace.")
        ui.dim("  Make some changes first, then summon again.\n")
        return 0
    import re
    n_files = len(re.findall(r"^diff --git", diff, re.M))
    ui.dim(f"  Branch: {branch or 'unknown'}\n  Changed files: {n_files}")
    preview = diff[:500].replace("\n", " ").strip()
    topic = (f'Review de huidige wijzigingen op branch "{branch or "unknown"}". {n_files} bestand(en) gewijzigd. '
             f"Diff preview: {preview}")
    ui.print("\n  The knights shall review your changes...\n", "bold")
    return discuss(topic, args, ui)


# ---- read-only views ----------------------------------------------------------------------------
PHASES = {"discussing": ("⚔️", "debating", "Discussing — swords are drawn"),
          "consensus_reached": ("✅", "consensus", "Consensus — ready to apply"),
          "escalated": ("⚠️", "escalated", "Escalated — the knights need your wisdom"),
          "applying": ("⚙️", "executing", "Applying — the knight is writing..."),
          "completed": ("✨", "done", "Completed — the deed is done")}


def cmd_status(args, ui: UI) -> int:
    s = store.find_latest_session(os.getcwd())
    if s is None:
        ui.warn("\n  The table is empty. No sessions yet.")
        ui.dim('  Run `roundtable discuss "topic"` to summon the knights.\n')
        return 0
    st = s.status or {}
    phase = st.get("phase", "unknown")
    ui.print("\n  Latest Session\n", "bold")
    ui.print(f"  Name:      {s.name}")
    ui.print(f"  Topic:     {s.topic or '—'}")
    ui.print(f"  Phase:     {PHASES.get(phase, ('', '', phase))[2]}")
    ui.print(f"  Round:     {st.get('round') or 0}")
    ui.print(f"  Consensus: {'Yes — miracles happen' if st.get('consensus_reached') else 'No — still arguing'}")
    for key, label in (("current_knight", "Knight:   "), ("lead_knight", "Lead:     "),
                       ("started_at", "Started:  "), ("updated_at", "Updated:  ")):
        if st.get(key):
            ui.print(f"  {label} {st[key]}")
    dp = os.path.join(s.path, "decisions.md")
    if os.path.exists(dp):
        with open(dp, encoding="utf-8") as f:
            content = f.read()
        ui.print("\n  The verdict:\n", "bold")
        ui.dim("\n".join(f"  {l}" for l in content.split("\n")[:10]))
        if len(content.split("\n")) > 10:
            ui.dim("  ...(the rest is in decisions.md)")
    ui.dim(f"\n  Path: {s.path}\n")
    return 0


def cmd_list(args, ui: UI) -> int:
    sessions = store.list_sessions(os.getcwd())
    if not sessions:
        ui.warn("\n  No battles fought yet.")
        ui.dim('  Run `roundtable discuss "topic"` to start one.\n')
        return 0
    ui.print(f"\n  The Archives — {len(sessions)} session(s)\n", "bold")
    for s in sessions:
        phase = (s.status or {}).get("phase", "unknown")
        icon, label, _ = PHASES.get(phase, ("?", phase, phase))
        rnd = (s.status or {}).get("round") or 0
        topic = s.topic or "—"
        if len(topic) > 60:
            topic = topic[:57] + "..."
        ui.print(f"  {icon} {label:<12} {s.name}")
        ui.print(f"    {topic} ({rnd} round{'' if rnd == 1 else 's'})\n")
    return 0


def cmd_chronicle(args, ui: UI) -> int:
    import re
    root = os.getcwd()
    path = ".roundtable/chronicle.md"
    try:
        path = load_config(root).chronicle
    except ConfigError as e:
        if "No .roundtable/config.json found" not in e.message:
            raise
    content = store.read_chronicle(root, path)
    if not content.strip():
        ui.warn("\n  The chronicle is blank. No decisions recorded yet.")
        ui.dim("  Win some debates first, then come back.\n")
        return 0
    n = len(re.findall(r"^## \d{4}", content, re.M))
    ui.print(f"\n  The Chronicle — {n} decision(s) etched in stone\n", "bold")
    ui.dim("  " + "=" * 56)
    for line in content.split("\n"):
        if line.startswith("# "):
            ui.print(f"  {line}", "bold", "cyan")
        elif line.startswith("## "):
            ui.print(f"\n  {line}", "bold")
        elif line.startswith("---"):
            ui.dim("  " + "~" * 40)
        else:
            ui.print(f"  {line}")
    return 0


def cmd_decrees(args, ui: UI) -> int:
    log = store.read_decree_log(os.getcwd())
    if not log["entries"]:
        ui.dim("\n  No decrees yet. The King has spoken on nothing.\n")
        return 0
    ui.print("\n  King's Decree Log\n", "bold")
    for e in log["entries"]:
        rev = " [REVOKED]" if e.get("revoked") else ""
        ui.print(f"  {e['id']} {e['type'].upper()}{rev}")
        ui.dim(f"    Topic:   {e['topic']}\n    Reason:  {e['reason']}\n    Session: {e['session']}\n"
               f"    Date:    {e['date'][:10]}\n")
    active = sum(1 for e in log["entries"] if not e.get("revoked"))
    ui.dim(f"  Total: {len(log['entries'])} ({active} active, {len(log['entries']) - active} revoked)\n")
    return 0


def cmd_manifest(args, ui: UI) -> int:
    root = os.getcwd()
    if args.mcmd == "list":
        m = store.read_manifest(root)
        if not m["features"]:
            ui.dim("\n  The manifest is empty. No features tracked yet.")
            ui.dim("  Features are added automatically after `roundtable apply`.\n")
            return 0
        ui.print(f"\n  Implementation Manifest ({len(m['features'])} features)\n", "bold")
        from .store.manifest import status_icon
        for f in m["features"]:
            ui.print(f"  [{status_icon(f['status'])}] {f['id']} — {f.get('summary', '')}")
            ui.dim(f"      Status: {f['status']} | Knight: {f.get('lead_knight')} | {str(f.get('applied_at', ''))[:10]}")
            ui.dim(f"      Files: {', '.join(f.get('files', []))}")
            if f.get("files_skipped"):
                ui.warn(f"      Skipped: {', '.join(f['files_skipped'])}")
            if f.get("replaced_by"):
                ui.dim(f"      Replaced by: {f['replaced_by']}")
            ui.print("")
    elif args.mcmd == "add":
        if not args.feature_id or not args.files:
            ui.error("\n  Usage: roundtable manifest add <feature-id> --files file1.ts file2.ts\n")
            return 0
        summary = args.summary if args.summary is not None else ask(ui, "  Summary: ", "")
        from .utils.clock import iso_now
        store.add_manifest_entry(root, {"id": args.feature_id, "session": "manual", "status": "implemented",
                                        "files": args.files, "summary": summary.strip() or args.feature_id,
                                        "applied_at": iso_now(), "lead_knight": "manual"})
        ui.ok(f'\n  Added "{args.feature_id}" to manifest with {len(args.files)} file(s).\n')
    elif args.mcmd == "deprecate":
        if store.deprecate_feature(root, args.feature_id, args.replaced_by):
            ui.warn(f'\n  Deprecated "{args.feature_id}".')
            if args.replaced_by:
                ui.dim(f"  Replaced by: {args.replaced_by}")
        else:
            ui.error(f'\n  Feature "{args.feature_id}" not found in manifest.\n')
    elif args.mcmd == "check":
        w = store.check_manifest(root)
        if not w:
            ui.ok("\n  Manifest is consistent. All tracked files exist on disk.\n")
        else:
            ui.warn(f"\n  {len(w)} warning(s) found:\n")
            for x in w:
                ui.warn(f"    {x}")
    return 0


def cmd_apply(args, ui: UI) -> int:
    from .apply.apply import apply_command
    return apply_command(args, ui)


def cmd_code_red(args, ui: UI) -> int:
    from .codered import code_red_command
    return code_red_command(args, ui)


def cmd_bench(args, ui: UI) -> int:
    import subprocess
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(here, "bench.py")] + args.bench_args
    return subprocess.call(cmd)


def cmd_serve(args, ui: UI) -> int:
    tp = max(1, int(getattr(args, "tp", 1) or 1))
    if tp > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU of the tensor-parallel group, started before any GPU call
        from .parallel.launch import launch_ranks
        # (ROUNDTABLE_DIST_BACKEND=gloo: the rehearsal mode of parallel/cluster.py, ranks share GPUs)
        if args.device != "cpu" and os.environ.get("ROUNDTABLE_DIST_BACKEND", "").lower() != "gloo":
            import torch     # device_count() does not initialise the GPU on this image
            if torch.cuda.device_count() < tp:
                raise ConfigError(f"serve --tp {tp} needs {tp} GPUs, {torch.cuda.device_count()} visible",
                                  hint="Lower --tp, or run on a node with enough GPUs.")
        return launch_ranks(tp, list(getattr(args, "raw_argv", sys.argv[1:])), args.device == "cpu",
                            f"serve {args.model} tp={tp}")
    from .serve import build_server
    srv = build_server(args.model, weights=args.weights, device=args.device, dtype=args.dtype, host=args.host,
                       port=args.port, max_batch=args.max_batch or (64 if tp <= 1 else 16), max_tokens=args.max_tokens,
                       use_graphs=not args.no_graphs, num_blocks=args.num_blocks, tp=tp,
                       op_limit_s=float(args.op_timeout))
    if srv is None:            # a follower rank of serve --tp N: served rank 0 until shutdown
        return 0
    ui.ok(f"  ✓ {args.model} on {srv.engine.device}: {srv.engine.kv_capacity_tokens} KV tokens resident capacity")
    ui.dim(f"  serving {srv.url}/v1/chat/completions  (OpenAI)  and  {srv.url}/api/chat  (Ollama)")
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    finally:
        srv.close()
    return 0


# ---- parser -------------------------------------------------------------------------------------
def _discuss_flags(p):
    g = p.add_mutually_exclusive_group()
    g.add_argument("--read-codebase", dest="read_codebase", action="store_true", default=None)
    g.add_argument("--no-read-codebase", dest="read_codebase", action="store_false")
    p.add_argument("--round-mode", choices=["sequential", "parallel"])
    p.add_argument("--layout", choices=["reference", "append"])
    p.add_argument("--max-new-tokens", type=int)
    p.add_argument("--seed", type=int, help="seed the speaking-order shuffle (default: unseeded)")
    p.add_argument("--choice", type=int, help="non-interactive King's choice when no consensus")
    p.add_argument("--decree", choices=["self", "later", "reject"], help="King's decree after consensus")
    p.add_argument("--decree-reason", default=None)
    p.add_argument("--resume", help="continue a session from its rounds.jsonl ('latest' or a session name)")
    p.add_argument("--device", help="force every knight onto this device (e.g. cpu, cuda:0)")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="roundtable", description="TheRoundtAIble — Where no AI is King, but all serve the Code. (MI355X engine)")
    p.add_argument("--version", action="version", version=__version__)
    p.add_argument("--quiet", action="store_true")
    sub = p.add_subparsers(dest="cmd", required=True)
    i = sub.add_parser("init", help="Initialize TheRoundtAIble in the current project")
    i.add_argument("--yes", "-y", action="store_true", help="accept defaults non-interactively")
    i.add_argument("--project")
    i.add_argument("--language")
    i.add_argument("--model", default="llama3-8b")
    i.add_argument("--weights", default="random:0")
    i.add_argument("--knights", type=int, default=3)
    i.add_argument("--tp", type=int, default=None,
                   help="tensor-parallel degree for every knight (default: automatic placement from the GPU scout)")
    i.add_argument("--placement", choices=["auto", "spread", "pack"], default="auto",
                   help="automatic placement policy: auto = measured cost model (fastest predicted round), "
                        "spread = one knight per GPU group, pack = same-model knights on one group")
    i.add_argument("--max-new-tokens", type=int, default=512)
    i.add_argument("--local-models", action="store_true",
                   help="seat every detected local checkpoint (ROUNDTABLE_MODELS_DIR, ./models, HF cache)")
    i.add_argument("--servers", action="store_true",
                   help="seat models of running LM Studio (:1234) / Ollama (:11434) servers over HTTP")
    i.add_argument("--external-clis", action="store_true",
                   help="seat installed claude/gemini/codex CLIs on their own transport instead of the engine")
    i.set_defaults(fn=cmd_init)
    d = sub.add_parser("discuss", help="Start a discussion between knights")
    d.add_argument("topic")
    _discuss_flags(d)
    d.set_defaults(fn=cmd_discuss)
    s = sub.add_parser("summon", help="Start a discussion based on current git diff")
    _discuss_flags(s)
    s.set_defaults(fn=cmd_summon)
    a = sub.add_parser("apply", help="Execute the consensus decision (lead knight writes code)")
    a.add_argument("--noparley", action="store_true", help="write without file-by-file review")
    a.add_argument("--dry-run", action="store_true", help="run the full pipeline without writing files")
    a.add_argument("--override-scope", action="store_true", help="bypass scope enforcement (requires a reason)")
    a.add_argument("--reason", help="override-scope reason (non-interactive)")
    a.add_argument("--yes", action="store_true", help="accept every parley prompt")
    a.add_argument("--session", help="session name (default: latest)")
    a.add_argument("--max-new-tokens", type=int)
    a.add_argument("--device")
    a.add_argument("--response-file", help="use this file as the lead knight's edit output (testing)")
    a.set_defaults(fn=cmd_apply)
    for name, fn, h in (("status", cmd_status, "Show the status of the latest discussion"),
                        ("list", cmd_list, "List all discussion sessions"),
                        ("chronicle", cmd_chronicle, "View the decision log"),
                        ("decrees", cmd_decrees, "View the King's Decree Log")):
        sub.add_parser(name, help=h).set_defaults(fn=fn)
    cr = sub.add_parser("code-red", help="Emergency diagnostic mode (triage, blind round, convergence)")
    cr.add_argument("symptoms")
    _discuss_flags(cr)
    cr.set_defaults(fn=cmd_code_red)
    m = sub.add_parser("manifest", help="Manage the implementation manifest")
    msub = m.add_subparsers(dest="mcmd", required=True)
    msub.add_parser("list")
    ma = msub.add_parser("add")
    ma.add_argument("feature_id")
    ma.add_argument("--files", nargs="+", default=[])
    ma.add_argument("--summary")
    md = msub.add_parser("deprecate")
    md.add_argument("feature_id")
    md.add_argument("--replaced-by")
    msub.add_parser("check")
    m.set_defaults(fn=cmd_manifest)
    sv = sub.add_parser("serve", help="Host a knight model behind an OpenAI/Ollama-compatible HTTP endpoint")
    sv.add_argument("--model", default="llama3-8b")
    sv.add_argument("--weights", default="random:0", help="random:<seed> | random-full:<seed> | <safetensors dir>")
    sv.add_argument("--device", default="cuda:0")
    sv.add_argument("--dtype", default="bf16")
    sv.add_argument("--host", default="127.0.0.1")
    sv.add_argument("--port", type=int, default=8000)
    sv.add_argument("--max-batch", type=int, default=None,
                    help="requests decoded together (default 64 at tp 1: 64 clients 6.4K -> 8.2K tok/s over "
                         "32, profiles/r06/serve; 16 with --tp: the rows the fused TP decode path takes)")
    sv.add_argument("--max-tokens", type=int, default=512, help="default completion budget per request")
    sv.add_argument("--num-blocks", type=int, default=None, help="KV blocks (default: sized from free memory)")
    sv.add_argument("--no-graphs", action="store_true")
    sv.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree: serve one model over N GPUs (N ranks; rank 0 serves HTTP)")
    sv.add_argument("--op-timeout", type=float, default=660.0,
                    help="--tp: seconds one engine operation may take on any rank; a rank past it (or one that "
                         "raises) ends the server with a message naming it (collectives time out a minute later)")
    sv.set_defaults(fn=cmd_serve)
    b = sub.add_parser("bench", help="Run the roundtable benchmark (wraps bench.py)")
    b.add_argument("bench_args", nargs=argparse.REMAINDER)
    b.set_defaults(fn=cmd_bench)
    return p


def _update_notice(ui: UI) -> None:
    """index.ts:185: print a notice when a newer version exists (opt-in, utils/update_check.py)."""
    from .utils.update_check import check_for_update
    latest = check_for_update()
    if latest:
        ui.warn(f"\n  Update available: {__version__} -> {latest}")


def main(argv: Optional[List[str]] = None) -> int:
    from .utils.debug import apply_debug_env
    apply_debug_env()          # ROUNDTABLE_DEBUG=1: serialized kernels + paging guards (before any HIP call)
    raw_argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    args.raw_argv = raw_argv
    ui = UI(quiet=args.quiet)
    try:
        if args.fn in (cmd_discuss, cmd_summon, cmd_apply, cmd_code_red):
            # a knight placement with tp > 1 needs one process per GPU: re-run this command as a
            # child torchrun BEFORE anything touches a GPU (parallel/launch.py)
            from .parallel.launch import maybe_relaunch
            rc = maybe_relaunch(raw_argv, quiet=args.quiet)
            if rc is not None:
                return rc
        rc = int(args.fn(args, ui) or 0)
        _update_notice(ui)
        return rc
    except RoundtableError as e:
        print(format_error(e), file=sys.stderr)
        return int(e.exit_code)
    except KeyboardInterrupt:
        return 130
    except Exception as e:  # noqa: BLE001 - the single error sink
        print(f"\n  Unexpected error: {e}", file=sys.stderr)
        if os.environ.get("DEBUG"):
            import traceback
            traceback.print_exc()
        return get_exit_code(e)
    finally:
        from .utils import failsafe
        g = failsafe.guard()
        if g is not None:
            g.finish()


if __name__ == "__main__":
    sys.exit(main())
