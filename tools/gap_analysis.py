#!/usr/bin/env python3
"""Idle time between consecutive kernels of a rocprofv3 --kernel-trace run (one GPU, one queue
at a time): where the GPU waits between launches, grouped by (previous kernel, next kernel).

Usage: gap_analysis.py <prof_dir> [out.md]
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    m = re.match(r"([A-Za-z_0-9]+)(<[^>]*>)?", n)
    base = m.group(1) if m else n[:40]
    if base.startswith("Cijk"):
        return "hipblaslt_gemm"
    return base + (m.group(2) if m and m.group(2) and len(m.group(2)) < 24 else "")


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    with open(paths[0]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    gaps = collections.defaultdict(list)
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    big = 0
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = s1 - e0
        if g > 200_000:      # > 200 us: host work between turns / rounds, reported apart
            big += g
            continue
        gaps[(n0, n1)].append(g)
    small = sum(sum(v) for v in gaps.values())
    lines = [f"kernels {len(rows)}, span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, "
             f"gaps <= 200 us: {small / 1e6:.1f} ms, gaps > 200 us (host phases): {big / 1e6:.1f} ms", "",
             "| previous -> next | count | mean gap us | total ms |", "|---|---|---|---|"]
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:30]:
        lines.append(f"| {a} -> {b} | {len(v)} | {sum(v) / len(v) / 1e3:.2f} | {sum(v) / 1e6:.2f} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
