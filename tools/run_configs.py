#!/usr/bin/env python3
"""Run the BASELINE.md configurations end to end and print one JSON line each.

    python tools/run_configs.py --config 1        # CPU plumbing: 2-knight GPT-2-small discuss via the CLI
    python tools/run_configs.py --config 3        # 8-knight Mistral-7B discuss, max_rounds=5 (bench.py)
    python tools/run_configs.py --config 4        # 3-knight summon on a synthetic git diff + apply --dry-run
    python tools/run_configs.py --config 2        # = bench.py defaults (the headline metric)

Config 5 (2 knights of Llama-3-70B at TP=4) needs 8 GPUs: ``torchrun --nproc-per-node 8
bench.py --model llama3-70b --tp 4 --knights-per-table 2``; it is not launched from here.

All knights use random-init weights and synthetic inputs (no checkpoints, no network);
EOS is ignored at a fixed ``max_new_tokens`` so every round runs to ``max_rounds``
(BASELINE.md measurement protocol). Wall-clock is measured around the CLI call.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def _config(knights, engine, rules_extra=None):
    rules = {"max_rounds": 1, "consensus_threshold": 9, "timeout_per_turn_seconds": 3600,
             "escalate_to_user_after": 9, "auto_execute": False, "ignore": [".git", "node_modules"]}
    rules.update(rules_extra or {})
    return {"version": "1.0", "project": "synthetic", "language": "nl", "knights": knights, "rules": rules,
            "chronicle": ".roundtable/chronicle.md", "adapter_config": {}, "engine": engine}


def _write_project(root, cfg):
    os.makedirs(os.path.join(root, ".roundtable", "sessions"), exist_ok=True)
    with open(os.path.join(root, ".roundtable", "config.json"), "w") as f:
        json.dump(cfg, f, indent=2)
    with open(os.path.join(root, ".roundtable", "chronicle.md"), "w") as f:
        f.write("# Chronicle\n")


def _session_metrics(root):
    from theroundtaible_amd import store
    sessions = store.list_sessions(root)
    path = sessions[0].path if sessions else None
    rows = []
    if path and os.path.exists(os.path.join(path, "metrics.jsonl")):
        with open(os.path.join(path, "metrics.jsonl")) as f:
            rows = [json.loads(line) for line in f if line.strip()]
    return path, rows


def config1():
    """2-knight discuss, GPT-2-small on CPU, max_rounds=1 — through the real CLI."""
    from theroundtaible_amd.cli import main
    root = tempfile.mkdtemp(prefix="rt-cfg1-")
    knights = [{"name": n, "adapter": f"local-llm-{n.lower()}", "capabilities": ["x"], "priority": i + 1}
               for i, n in enumerate(["Alfa", "Beta"])]
    _write_project(root, _config(knights, {"default_model": "gpt2-small", "weights": "random:1", "device": "cpu",
                                           "max_new_tokens": 32, "ignore_eos": True}))
    cwd = os.getcwd()
    os.chdir(root)
    try:
        t0 = time.perf_counter()
        rc = main(["--quiet", "discuss", "Plumbing-test van de rondetafel", "--no-read-codebase",
                   "--device", "cpu", "--choice", "3"])
        wall = time.perf_counter() - t0
    finally:
        os.chdir(cwd)
    return {"config": 1, "desc": "2-knight discuss, GPT-2-small, CPU, max_rounds=1", "rc": rc,
            "wall_s": round(wall, 3), "ms_per_round": round(wall * 1e3, 1), "device": "cpu"}


def _bench(extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        raise RuntimeError(f"bench failed rc={r.returncode}: {r.stderr[-2000:]}")
    return json.loads(line[-1])


def config2(steps):
    out = _bench(["--steps", str(steps), "--warmup", "1"])
    return {"config": 2, "desc": "3-knight discuss, Llama-3-8B bf16 (bench.py headline)", **out}


def config3(steps):
    out = _bench(["--model", "mistral-7b", "--knights-per-table", "8", "--knights-per-gpu", "8",
                  "--steps", str(steps), "--warmup", "1"])
    return {"config": 3, "desc": f"8-knight discuss, Mistral-7B, {steps + 1} rounds, all knights batched per GPU",
            **out}


SRC_TEMPLATE = '''"""Synthetic module {i}: cache layer shard {i}."""
from dataclasses import dataclass


@dataclass
class Entry{i}:
    key: str
    value: bytes
    ttl: int = 60


class Shard{i}:
    def __init__(self, capacity: int = {cap}):
        self.capacity = capacity
        self.items = {{}}

    def get(self, key):
        e = self.items.get(key)
        return None if e is None else e.value

    def put(self, key, value, ttl=60):
        if len(self.items) >= self.capacity:
            self.evict()
        self.items[key] = Entry{i}(key, value, ttl)

    def evict(self):
        oldest = min(self.items.values(), key=lambda e: e.ttl)
        del self.items[oldest.key]
'''


def config4(files: int, new_tokens: int, model: str = "llama3-8b", scripted: bool = True):
    """3-knight summon over a synthetic git diff with the codebase read (long context), then apply --dry-run.

    ``scripted`` (default): the knights' replies end in the forced consensus tail (knights/script.py),
    so the table agrees in round 1 and ``apply --dry-run`` plans the lead knight's RTDIFF/1 edit
    (random weights alone never write a parseable block); the ``shared`` layout keeps one copy of
    the ~11K-token summon context's KV for the three knights."""
    from theroundtaible_amd.cli import main
    root = tempfile.mkdtemp(prefix="rt-cfg4-")
    src = os.path.join(root, "src")
    os.makedirs(src)
    for i in range(files):
        with open(os.path.join(src, f"shard_{i:03d}.py"), "w") as f:
            f.write(SRC_TEMPLATE.format(i=i, cap=64 + i))
    git = ["git", "-c", "user.email=bench@example.invalid", "-c", "user.name=bench"]
    subprocess.run(git + ["init", "-q"], cwd=root, check=True)
    subprocess.run(git + ["add", "-A"], cwd=root, check=True)
    subprocess.run(git + ["commit", "-qm", "synthetic base"], cwd=root, check=True)
    for i in range(0, files, 7):   # the diff under review
        p = os.path.join(src, f"shard_{i:03d}.py")
        with open(p) as f:
            s = f.read()
        with open(p, "w") as f:
            f.write(s.replace("min(self.items.values(), key=lambda e: e.ttl)",
                              "min(self.items.values(), key=lambda e: (e.ttl, e.key))"))
    knights = [{"name": n, "adapter": a, "capabilities": ["x"], "priority": i + 1}
               for i, (n, a) in enumerate([("Claude", "claude-cli"), ("Gemini", "gemini-cli"), ("GPT", "openai-cli")])]
    engine = {"default_model": model, "weights": "random:3", "max_new_tokens": new_tokens, "ignore_eos": True}
    if scripted:
        engine["scripted_consensus"] = {"free_tokens": new_tokens, "scores": [9], "files": ["NEW:docs/besluit.md"]}
    _write_project(root, _config(knights, engine, {"prompt_layout": "shared"}))
    cwd = os.getcwd()
    os.chdir(root)
    try:
        t0 = time.perf_counter()
        rc1 = main(["--quiet", "summon", "--read-codebase", "--choice", "1"])
        t1 = time.perf_counter()
        rc2 = main(["--quiet", "apply", "--dry-run", "--yes"])
        t2 = time.perf_counter()
    finally:
        os.chdir(cwd)
    path, rows = _session_metrics(root)
    prompt_tokens = sum(int(r.get("prefill_tokens", 0)) + int(r.get("reused_tokens", 0)) for r in rows)
    plan = None
    if path and os.path.exists(os.path.join(path, "apply-plan.json")):
        with open(os.path.join(path, "apply-plan.json")) as f:
            p = json.load(f)
        plan = {"planned": [x["path"] for x in p["planned"]], "skipped": p["skipped"]}
    return {"config": 4, "desc": f"3-knight summon (synthetic diff, --read-codebase) + apply --dry-run, {model}",
            "scripted_consensus": scripted, "apply_plan": plan,
            "rc_summon": rc1, "rc_apply": rc2, "summon_s": round(t1 - t0, 3), "apply_dry_run_s": round(t2 - t1, 3),
            "source_files": files, "turn_metrics": rows[-3:] if rows else [], "prompt_tokens_total": prompt_tokens}


def main_():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True, choices=[1, 2, 3, 4])
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--files", type=int, default=120, help="config 4: synthetic source files read into context")
    ap.add_argument("--new-tokens", type=int, default=256)
    ap.add_argument("--model", default="llama3-8b", help="config 4 model (tiny-llama for a CPU smoke run)")
    ap.add_argument("--no-script", action="store_true", help="config 4: free replies only (no forced consensus)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {1: config1, 2: lambda: config2(a.steps), 3: lambda: config3(a.steps),
           4: lambda: config4(a.files, a.new_tokens, a.model, not a.no_script)}[a.config]()
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main_())
