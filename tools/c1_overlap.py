#!/usr/bin/env python3
"""C1 / speculative-prefill overlap from a striped multi-rank run (VERDICT r2 #6 evidence).

Inputs per rank: the pool's event log (``bench.py --c1-events <path>`` -> ``<path>.r<rank>.json``:
c1_start / speculate / speculate_end / c1_wait with CLOCK_MONOTONIC ns) and that rank's
``rocprofv3 --kernel-trace --output-format csv`` directory (same clock). For every C1 exchange
(c1_start -> c1_wait) it reports how long the exchange was in flight and which GPU kernels ran
inside that window — the speculative prefill of the next round's known prefix.

    python tools/c1_overlap.py <events-prefix> <trace-dir-rank0> [<trace-dir-rank1> ...] > out.md
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys


def kernels(trace_dir):
    out = []
    for path in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                try:
                    out.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row.get("Kernel_Name", "?")))
                except (KeyError, ValueError):
                    continue
    out.sort()
    return out


def windows(ev):
    names, ns = ev["events"], ev["ns"]
    res, cur = [], None
    for n, t in zip(names, ns):
        if n == "c1_start":
            cur = {"start": t, "spec": None, "spec_end": None}
        elif cur is not None and n == "speculate" and cur["spec"] is None:
            cur["spec"] = t
        elif cur is not None and n == "speculate_end":
            cur["spec_end"] = t
        elif cur is not None and n == "c1_wait":
            cur["wait"] = t
            res.append(cur)
            cur = None
    return res


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    for sep in ("<", "("):
        name = name.split(sep)[0]
    return name[:40]


def main(argv):
    prefix, dirs = argv[0], argv[1:]
    print("# C1 all-gather overlapped with the speculative prefill (2-rank striped rehearsal)\n")
    print("Per exchange: C1 in flight from `ex.start` (async all-gather issued) to `ex.wait` returning; "
          "GPU kernels of THIS rank that executed inside that window (they were enqueued by the "
          "speculative prefill of the next round's known prefix, `Engine.warm_shared`).\n")
    for r, d in enumerate(dirs):
        ev = json.load(open(f"{prefix}.r{r}.json"))
        ks = kernels(d)
        print(f"## rank {r}\n")
        print("| exchange | C1 in flight (ms) | speculated | kernels inside window | GPU busy inside window (ms) | top kernels |")
        print("|---|---|---|---|---|---|")
        tot_w = tot_b = 0.0
        for i, w in enumerate(windows(ev)):
            a, b = w["start"], w["wait"]
            inside = [(s, e, n) for s, e, n in ks if s < b and e > a]
            busy = sum(min(e, b) - max(s, a) for s, e, _ in inside) / 1e6
            names = {}
            for s, e, n in inside:
                names[short(n)] = names.get(short(n), 0) + 1
            top = ", ".join(f"{k} x{v}" for k, v in sorted(names.items(), key=lambda x: -x[1])[:3])
            spec = "yes" if w["spec"] is not None else "no"
            tot_w += (b - a) / 1e6
            tot_b += busy
            print(f"| {i} | {(b - a) / 1e6:.2f} | {spec} | {len(inside)} | {busy:.2f} | {top} |")
        print(f"\nrank {r}: {tot_b:.1f} ms of GPU work ran inside {tot_w:.1f} ms of C1 exchange windows\n")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
