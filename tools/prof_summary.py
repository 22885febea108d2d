#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace --stats run into a small markdown table.

Usage: prof_summary.py <prof_dir> <out.md> [--drop-trace]
Reads <prefix>_kernel_stats.csv (+ kernel_trace.csv for per-dispatch VGPR/LDS/grid info),
or, when rocprofv3 wrote its default rocpd SQLite output (``*_results.db``), the ``kernels``
view of that database; writes the top kernels by total time, and optionally deletes the (large) trace CSV so the
gpurun_out/ payload stays small.
"""
import csv
import glob
import os
import sys


def from_db(path):
    """Aggregate the rocpd ``kernels`` view into the same row/info shape as the CSV path."""
    import sqlite3
    con = sqlite3.connect(path)
    rows, info = [], {}
    q = ("select name, count(*), sum(duration), avg(duration), max(vgpr_count), max(accum_vgpr_count), "
         "max(sgpr_count), max(lds_size), max(scratch_size), max(workgroup_x), max(grid_x), max(grid_y) "
         "from kernels group by name")
    for (n, calls, tot, avg, v, a, s, lds, scr, wg, gx, gy) in con.execute(q):
        rows.append({"Name": n, "Calls": calls, "TotalDurationNs": tot, "AverageNs": avg})
        info[n] = {"VGPR_Count": v, "Accum_VGPR_Count": a, "SGPR_Count": s, "LDS_Block_Size": lds,
                   "Scratch_Size": scr, "Workgroup_Size_X": wg, "Grid_Size_X": gx, "Grid_Size_Y": gy}
    con.close()
    return rows, info


def main():
    d, out = sys.argv[1], sys.argv[2]
    drop = "--drop-trace" in sys.argv
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dbs = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)
    rows = []
    if not stats and dbs:
        rows, info = from_db(dbs[0])
        return write(rows, info, out, [], drop)
    if stats:
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                rows.append(r)
    info = {}
    if trace:
        with open(trace[0]) as f:
            for r in csv.DictReader(f):
                n = r.get("Kernel_Name", "")
                if n not in info:
                    info[n] = {k: r.get(k, "") for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                                         "LDS_Block_Size", "Scratch_Size", "Workgroup_Size_X",
                                                         "Grid_Size_X", "Grid_Size_Y")}
    return write(rows, info, out, trace, drop)


def write(rows, info, out, trace, drop):
    total = sum(float(r.get("TotalDurationNs", 0) or 0) for r in rows) or 1.0
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
    lines = ["| kernel | calls | total ms | avg us | % | VGPR | AGPR | LDS | grid x,y | wg |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows[:40]:
        name = r.get("Name", r.get("KernelName", ""))
        i = info.get(name, {})
        short = name if len(name) < 90 else name[:87] + "..."
        tot = float(r.get("TotalDurationNs", 0) or 0)
        lines.append(f"| `{short}` | {r.get('Calls')} | {tot / 1e6:.2f} | {float(r.get('AverageNs', 0) or 0) / 1e3:.1f} "
                     f"| {100 * tot / total:.1f} | {i.get('VGPR_Count', '')} | {i.get('Accum_VGPR_Count', '')} "
                     f"| {i.get('LDS_Block_Size', '')} | {i.get('Grid_Size_X', '')},{i.get('Grid_Size_Y', '')} "
                     f"| {i.get('Workgroup_Size_X', '')} |")
    lines.append(f"\nTotal kernel time: {total / 1e6:.1f} ms over {sum(int(r.get('Calls', 0) or 0) for r in rows)} dispatches")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:30]))
    if drop:
        for t in trace:
            os.remove(t)


if __name__ == "__main__":
    main()
