#!/usr/bin/env python3
"""Predicted strong-scaling curve of the headline bench (ONE 3-knight Llama-3-8B table, engine
tensor-parallel over N GPUs) from single-GPU measurements — VERDICT r2 next #1's cost model.

Per rank, a round = the rank's own compute + the collectives it waits for:

* compute: ``bench.py --simulate-tp N`` on ONE MI355X runs rank 0's exact shard (split-K shard
  GEMMs, 1/N of the KV heads in the grouped decode attention, vocab-sharded lm_head, the
  captured decode graph, the real orchestrator) with every collective elided
  (parallel/tp.py SimulatedTP): ``engine_decode_ms_per_round`` + prefill + host time;
* decode collectives per step: 2 x n_layers K9 one-shot all-reduces ([3, 4096] bf16) + one
  vocab-parallel logits all-gather; K9's kernel cost was measured between ranks sharing one GPU
  (tools/oneshot_check.py --bench); the xGMI hop is NOT measurable on a 1-GPU box, so the curve
  is printed for a range of per-call latencies;
* prefill collectives per round: 2 x n_layers RCCL ring all-reduces of [new tokens, 4096] bf16
  (bus bandwidth estimate, parallel/costmodel.py Calibration.prefill_ar_gbps).

    python tools/tp_cost.py profiles/r03/sim{1,2,4,8}.json > profiles/r03/tp_cost_model.md
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(paths) -> int:
    from theroundtaible_amd.models.config import get_config
    from theroundtaible_amd.parallel.costmodel import Calibration, strong_round_ms
    sims, dev = {}, {}
    for p in paths:
        d = json.load(open(p))
        # records with device-simulated collectives (bench.py --simulate-tp N --sim-k9-us X, round 5)
        # are the model's check, not its input
        (dev if (d["detail"].get("sim_comm") or None) else sims)[int(d["config"]["tp"])] = d
    base = sims.get(1)
    if base is None:
        raise SystemExit("need the tp=1 run (sim1.json)")
    cfg = get_config("llama3-8b")
    cal = Calibration()
    L = cfg.n_layers
    mode = base["config"].get("round_mode", "parallel")
    turns = base["config"]["knights_per_table"] if mode == "sequential" else 1
    steps = base["config"]["new_tokens_per_turn"] * turns
    rounds = base["steps"]
    pre_tok = base["detail"]["prefill_tokens"] / rounds          # new tokens prefilled per round (all knights)
    dec_tok = base["detail"]["decode_tokens"] / rounds
    print(f"# Strong-scaling cost model: one 3-knight Llama-3-8B table on a tp=N engine ({mode} rounds)\n")
    how = "3 knights batched" if mode == "parallel" else "the 3 speakers one after another, B = 1"
    print(f"Workload = the driver's bench config: {rounds} timed rounds, {steps} decode steps per round "
          f"({how}), {pre_tok:.0f} prefill tokens per round, shared layout, {mode} rounds.\n")
    print("Per-rank compute measured on ONE MI355X with `bench.py --simulate-tp N` (rank 0's exact shard, "
          "collectives elided); collectives added from the per-call latencies below.\n")
    print("| N | compute ms/round (measured) | decode ms/step (measured) | prefill AR ms/round | "
          + " | ".join(f"K9 {us} us: ms/round (tok/s)" for us in (5, 8, 12, 20)) + " |")
    print("|---|---|---|---|" + "---|" * 4)
    for n in sorted(sims):
        d = sims[n]
        comp = d["ms_per_round"]
        dstep = d["detail"]["engine_decode_ms_per_round"] / steps
        # the prefill ring all-reduces alone = the prediction with free decode collectives
        par = strong_round_ms(d, n, 0.0, 0.0, cal=cal) - comp
        cells = []
        for us in (5, 8, 12, 20):
            tot = strong_round_ms(d, n, us, cal.gather_us, cal=cal)
            cells.append(f"{tot:.0f} ({dec_tok / tot * 1e3:.0f})")
        print(f"| {n} | {comp:.0f} | {dstep:.3f} | {par:.1f} | " + " | ".join(cells) + " |")
    if dev:
        print("\nCheck of the additive model against the DEVICE-simulated collectives (round 5: `bench.py "
              "--simulate-tp N --sim-k9-us X` — every all-reduce / gather is a kernel holding the K9 launch's CUs "
              "for X us inside the captured graph, so the step pays it on the stream as a node would):\n")
        print("| N | all-reduce us | compute-only decode ms/step | device-simulated decode ms/step | "
              "additive model decode ms/step | device-simulated ms/round (tok/s) |")
        print("|---|---|---|---|---|---|")
        for n in sorted(dev):
            d, c = dev[n], sims.get(n)
            sc = d["detail"]["sim_comm"]
            dd = d["detail"]["engine_decode_ms_per_round"] / steps
            cc = c["detail"]["engine_decode_ms_per_round"] / steps if c else float("nan")
            model = cc + (2 * L * sc["all_reduce_us"] + sc["gather_us"]) / 1e3
            print(f"| {n} | {sc['all_reduce_us']:g} | {cc:.3f} | {dd:.3f} | {model:.3f} | "
                  f"{d['ms_per_round']:.0f} ({d['value']:.0f}) |")
        print("\n(The device stand-in charges a prefill all-reduce the same per-call latency; the additive "
              "model's prefill column charges the RCCL ring bandwidth instead.)")
    print("\nK9 per call measured between ranks sharing one GPU (IPC, no xGMI hop): "
          "5.4 us (2 ranks, 16 KB) — tools/oneshot_check.py --bench, profiles/r03/k9_shared_gpu.log.")
    print(f"Logits gather per step: {cal.gather_us} us (K9 one-shot all-gather, 2 ranks sharing one GPU, "
          "profiles/r03/k9_fused_gather_shared_gpu.md).")
    print("The driver's 8-GPU run (SCALE_rNN.json) confirms or refutes the column that matches the real xGMI latency; "
          "its bench detail carries the node's own K9 latency (`k9_us`, measured at engine creation) and the "
          "measured per-call saving of the fused GEMM + all-reduce (`k9_fused_saving_us`, used when > 0.5 us: "
          "subtract it from the K9 column).")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
