#!/usr/bin/env python3
"""GPU idle-time analysis of a rocprofv3 kernel trace: where the device waits on the host.

    python tools/gpu_idle.py gpurun_out/prof [--min-gap-us 20] [--last-ms 4000]

Sorts dispatches by start time, sums busy time (union of kernel intervals) and the gaps
between them over the analysed window (by default the whole trace; ``--last-ms`` keeps the
final N ms, e.g. the timed rounds of bench.py), and lists the largest gaps with the kernels
on either side — a gap after the last kernel of a decode step is graph-replay / host latency,
one after an lm_head of a prefill is orchestration / tokenisation.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--min-gap-us", type=float, default=20.0)
    ap.add_argument("--last-ms", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    rows.sort()
    if a.last_ms > 0:
        t_end = max(e for _, e, _ in rows)
        rows = [r for r in rows if r[0] >= t_end - a.last_ms * 1e6]
    busy = 0
    gaps = []
    cur_s, cur_e, prev_name = rows[0][0], rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    idle = sum(g for g, _, _ in gaps)
    big = [g for g in gaps if g[0] >= a.min_gap_us * 1e3]
    print(f"window {span / 1e6:.1f} ms, {len(rows)} dispatches: busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms "
          f"({100 * idle / span:.1f} %); gaps >= {a.min_gap_us:g} us: {len(big)} totalling "
          f"{sum(g for g, _, _ in big) / 1e6:.1f} ms")
    small = [g for g in gaps if g[0] < a.min_gap_us * 1e3]
    if small:
        print(f"small gaps: {len(small)}, mean {sum(g for g, _, _ in small) / len(small) / 1e3:.2f} us")
    print("\n| gap us | after | before |\n|---|---|---|")
    for g, p, n in sorted(big, reverse=True)[:a.top]:
        print(f"| {g / 1e3:.1f} | `{p}` | `{n}` |")


if __name__ == "__main__":
    main()
