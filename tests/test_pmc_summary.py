"""tools/pmc_summary.py on synthetic rocprofv3 csv output (CPU)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_pmc_summary_joins_counters_with_durations(tmp_path):
    d = tmp_path / "pmc"
    d.mkdir()
    _write(d / "pmc_kernel_trace.csv", ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"],
           [[1, "gemm", 1000, 11000], [2, "gemm", 20000, 30000], [3, "attn", 40000, 45000]])
    # FETCH_SIZE is in KB: 1 GiB over 10 us per gemm call, 0.5 GiB over 5 us for attn
    _write(d / "pmc_counter_collection.csv", ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"],
           [[1, "gemm", "FETCH_SIZE", 1048576], [2, "gemm", "FETCH_SIZE", 1048576],
            [3, "attn", "FETCH_SIZE", 524288], [3, "attn", "OTHER", 7]])
    out = tmp_path / "s.md"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(d), str(out)],
                       capture_output=True, text=True, check=True)
    lines = out.read_text().splitlines()
    assert lines[0].startswith("| kernel | dispatches | mean FETCH_SIZE (MB)")
    gemm = next(l for l in lines if "`gemm`" in l).split("|")
    attn = next(l for l in lines if "`attn`" in l).split("|")
    assert gemm[2].strip() == "2" and gemm[3].strip() == "1024.00" and gemm[4].strip() == "10.00"
    assert int(gemm[5]) == 107374   # 1 GiB / 10 us in GB/s
    assert attn[2].strip() == "1" and attn[4].strip() == "5.00"
    assert lines.index(next(l for l in lines if "`gemm`" in l)) < lines.index(next(l for l in lines if "`attn`" in l))
    assert "gemm" in r.stdout
