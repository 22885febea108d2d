#!/usr/bin/env python3
"""Between-round (prefill) phase of a bench run from a rocprofv3 --kernel-trace: where the
~80 ms between one round's last decode step and the next round's first go.

Round boundaries are the long gaps between consecutive decode_advance launches (one per
captured decode step). For each boundary: GPU busy time by kernel, and the idle gaps (host
work: tokenisation, prompt build, first-token sampling, Python launch overhead).

Usage: prefill_phase.py <prof_dir> [out.md]
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from gap_analysis import short  # noqa: E402


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    adv = [i for i, r in enumerate(rows) if r[2].startswith("decode_advance")]
    bounds = [(a, b) for a, b in zip(adv, adv[1:]) if rows[b][0] - rows[a][1] > 20_000_000]
    lines = [f"kernels {len(rows)}, decode steps {len(adv)}, round boundaries {len(bounds)}", ""]
    for a, b in bounds[-3:]:
        # window: after the previous round's last step, up to the first kernel of the next
        # round's first captured step (the kernel after the eager decode_prep before b)
        j = b
        while j > a and not rows[j][2].startswith("decode_prep"):
            j -= 1
        end = rows[j + 1][0] if j > a else rows[b][0]
        win = [r for r in rows[a + 1:] if r[0] < end]
        span = end - rows[a][1]
        busy = collections.Counter()
        cnt = collections.Counter()
        for s, e, n in win:
            busy[n] += e - s
            cnt[n] += 1
        gaps = []
        prev_end, prev_name = rows[a][1], rows[a][2]
        for s, e, n in win:
            if s - prev_end > 50_000:
                gaps.append((s - prev_end, prev_name, n))
            prev_end, prev_name = max(prev_end, e), n
        if end - prev_end > 50_000:
            gaps.append((end - prev_end, prev_name, "next round decode"))
        tb = sum(busy.values())
        lines += [f"## boundary after step {adv.index(a)}: {span / 1e6:.1f} ms, kernels {len(win)}, "
                  f"GPU busy {tb / 1e6:.1f} ms, idle gaps > 50 us {sum(g for g, _, _ in gaps) / 1e6:.1f} ms", "",
                  "| kernel | count | busy ms |", "|---|---|---|"]
        for n, t in busy.most_common(14):
            lines.append(f"| {n} | {cnt[n]} | {t / 1e6:.2f} |")
        lines += ["", "| idle gap ms | after | before |", "|---|---|---|"]
        for g, p, n in sorted(gaps, reverse=True)[:12]:
            lines.append(f"| {g / 1e6:.2f} | {p} | {n} |")
        lines.append("")
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
