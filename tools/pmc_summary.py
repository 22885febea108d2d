#!/usr/bin/env python3
"""Per-kernel HBM traffic from a rocprofv3 counter pass (csv output).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir> -o pmc -- python tools/microbench.py ...
    python tools/pmc_summary.py <dir> <out.md> [--counter FETCH_SIZE]

Joins ``*_counter_collection.csv`` (one row per dispatch and counter) with
``*_kernel_trace.csv`` (start / end per dispatch) on the dispatch id and prints, per kernel
name: dispatches, mean counter value (FETCH_SIZE / WRITE_SIZE are in KB), mean duration and
the implied bandwidth. Deletes nothing; the csv files stay where rocprofv3 wrote them.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--counter", default="FETCH_SIZE")
    a = ap.parse_args()
    dur = {}
    for path in _find(a.dir, "kernel_trace.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                did = _col(r, "Dispatch_Id", "Correlation_Id")
                dur[did] = (int(_col(r, "End_Timestamp")) - int(_col(r, "Start_Timestamp"))) / 1e3
    acc = defaultdict(lambda: [0, 0.0, 0.0])   # name -> [n, counter sum, duration sum]
    for path in _find(a.dir, "counter_collection.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                if _col(r, "Counter_Name") != a.counter:
                    continue
                did = _col(r, "Dispatch_Id", "Correlation_Id")
                name = _col(r, "Kernel_Name")
                e = acc[name]
                e[0] += 1
                e[1] += float(_col(r, "Counter_Value"))
                e[2] += dur.get(did, 0.0)
    rows = sorted(acc.items(), key=lambda kv: -kv[1][1])
    lines = [f"| kernel | dispatches | mean {a.counter} (MB) | mean us | GB/s |", "|---|---|---|---|---|"]
    for name, (n, c, d) in rows:
        mb = c / n / 1024.0
        us = d / n if n else 0.0
        bw = (mb * 1024 * 1024 / 1e9) / (us / 1e6) if us > 0 else 0.0   # KB-based counter -> bytes
        short = name if len(name) <= 90 else name[:87] + "..."
        lines.append(f"| `{short}` | {n} | {mb:.2f} | {us:.2f} | {bw:.0f} |")
    text = "\n".join(lines) + "\n"
    with open(a.out, "w") as f:
        f.write(text)
    print(text)


if __name__ == "__main__":
    main()
