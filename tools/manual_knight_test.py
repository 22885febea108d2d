#!/usr/bin/env python3
"""Manual knight smoke test: one fixed JSON-echo prompt per adapter, latency + consensus parse.

Parity: `tests/manual-adapter-test.mjs:1-28` of the reference calls its three CLI adapters
with a prompt asking the model to echo a consensus block, prints the latency in ms and
checks for ``consensus_score: 9``. Here every adapter id resolves to an engine-hosted
model (see `knights/registry.py`), so the same check exercises model load, prefill,
decode and the consensus parser end to end.

    python tools/manual_knight_test.py                          # claude-cli, gemini-cli, openai-cli
    python tools/manual_knight_test.py --adapters fake engine-small --device cpu
    python tools/manual_knight_test.py --project /path/to/project   # use its .roundtable/config.json

With ``random:*`` weights the model cannot follow the instruction, so the parse check is
reported (not asserted) unless ``--strict`` is given; a ``fake`` adapter always passes.
Exit code: 0 when every adapter answered (and, with ``--strict``, echoed score 9).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from theroundtaible_amd.config import generate_config, load_config  # noqa: E402
from theroundtaible_amd.knights.fake import consensus_reply  # noqa: E402
from theroundtaible_amd.knights.registry import BackendFactory  # noqa: E402
from theroundtaible_amd.types import RoundtableConfig  # noqa: E402

PROMPT = ("Reply with ONLY this JSON block and nothing else:\n"
          '```json\n{"consensus_score": 9, "agrees_with": [], "pending_issues": []}\n```')


def _config(args) -> RoundtableConfig:
    if args.project:
        return load_config(args.project)
    eng = {"model": args.model, "weights": args.weights, "max_new_tokens": args.max_new_tokens,
           "temperature": 0.0, "use_graphs": False}
    if args.device:
        eng["device"] = args.device
    knights = [{"name": a, "adapter": a} for a in args.adapters]
    return RoundtableConfig.from_dict(generate_config("manual-knight-test", "en", knights, engine=eng))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--adapters", nargs="+", default=["claude-cli", "gemini-cli", "openai-cli"])
    ap.add_argument("--project", help="project root whose .roundtable/config.json to use")
    ap.add_argument("--model", default="tiny-llama")
    ap.add_argument("--weights", default="random:0")
    ap.add_argument("--device", default=None, help="cpu / cuda:N (default: auto placement)")
    ap.add_argument("--max-new-tokens", type=int, default=48)
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--strict", action="store_true", help="fail when a knight does not echo score 9")
    args = ap.parse_args(argv)

    cfg = _config(args)
    adapters = [k.adapter for k in cfg.knights] if args.project else args.adapters
    factory = BackendFactory(cfg)
    ok = True
    for aid in dict.fromkeys(adapters):
        try:
            be = factory.create(aid)
        except Exception as e:  # noqa: BLE001 - report and keep testing the others
            print(f"{aid}: FAILED to start ({e})")
            ok = False
            continue
        if be is None:
            print(f"{aid}: unknown adapter")
            ok = False
            continue
        if aid.startswith("fake"):
            be.script = lambda *_: consensus_reply(9)
        t0 = time.perf_counter()
        try:
            res = be.execute(PROMPT, args.timeout, seq_key=f"manual-{aid}", rnd=1)
        except Exception as e:  # noqa: BLE001
            print(f"{aid}: ERROR {type(e).__name__}: {e}")
            ok = False
            continue
        ms = (time.perf_counter() - t0) * 1000
        block = be.parse_consensus(res.text, 1)
        score = None if block is None else block.consensus_score
        echoed = score == 9
        ok &= echoed or not args.strict
        tps = res.metrics.get("decode_tokens")
        extra = f", {tps} decode tokens" if tps is not None else ""
        print(f"{aid} ({be.name}): {ms:.0f} ms{extra}, consensus_score={score} "
              f"[{'PASS' if echoed else 'no echo'}]")
        print("   " + res.text[:200].replace("\n", "\n   "))
        be.release(f"manual-{aid}")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
