"""Round-5 probe: the fused GEMM + all-reduce (EPI_AR) forced on at tp 4 / tp 8 with the ranks
sharing ONE GPU, each rank capped at GPU_MAX_HW_QUEUES queues, against tp 1 (tools/tp_check.py,
Llama-3-8B 2 layers, captured graphs): do the grids co-run and the results match?"""
import json
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nproc, queues=None, fused=False, extra=(), cu_split=False, ref_cus=None):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = os.path.join(ROOT, "gpurun_out", "r05p", f"tp{nproc}_q{queues}_f{int(fused)}_cu{int(cu_split)}_r{ref_cus}.pt")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tools", "tp_check.py"),
           "--model", "llama3-8b", "--layers", "2", "--tokens", "12", "--out", out, "--graphs", *extra]
    env = dict(os.environ, ROUNDTABLE_DIST_BACKEND="gloo", OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    if queues:
        env["GPU_MAX_HW_QUEUES"] = str(queues)
    if fused:
        env["ROUNDTABLE_FUSED_AR"] = "1"
    if cu_split:
        env["ROUNDTABLE_REHEARSAL_CU_SPLIT"] = "1"
    if ref_cus:      # a tp 1 reference on the same CU count as one rank of a split run
        env["ROC_GLOBAL_CU_MASK"] = hex((1 << ref_cus) - 1)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    if r.returncode != 0:
        print(r.stdout[-1500:], r.stderr[-3000:], flush=True)
        raise SystemExit(f"tp{nproc} q{queues} failed rc={r.returncode}")
    return torch.load(out, weights_only=True)


CASES = [(4, 4, False), (4, 2, False), (8, 2, False)]
if os.environ.get("CASES") == "cu":
    CASES = [(2, None, True), (4, None, True), (8, 2, True)]


def main():
    cos = torch.nn.functional.cosine_similarity
    for nproc, q, cu in CASES:
        # weights come from torch's device RNG, whose launch shapes follow the CU count a process
        # sees: a CU-split run is compared with a tp 1 run on one rank's slice
        ref = run(1, ref_cus=256 // nproc if cu else None)
        got = run(nproc, q, fused=True, extra=("--poll-limit", "262144"), cu_split=cu)
        errs = [e for e in got["errors"] if e is not None]
        row = {"tp": nproc, "queues_per_rank": q, "cu_split": cu, "fused_ar": got["fused_ar"], "fused_ar_calls": got["fused_ar_calls"],
               "graphs": all(got["graphs_per_rank"]), "errors": len(errs), "flag_errors": bool(got["flag_errors"]),
               "ids_equal_tp1": got["ids"] == ref["ids"],
               "decode_cos": round(float(cos(got["decode_logits"][None], ref["decode_logits"][None])), 6)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
