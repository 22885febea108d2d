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


def run(nproc, queues=None, fused=False, extra=()):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = os.path.join(ROOT, "gpurun_out", "r05p", f"tp{nproc}_q{queues}_f{int(fused)}.pt")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tools", "tp_check.py"),
           "--model", "llama3-8b", "--layers", "2", "--tokens", "12", "--out", out, "--graphs", *extra]
    env = dict(os.environ, ROUNDTABLE_DIST_BACKEND="gloo", OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    if queues:
        env["GPU_MAX_HW_QUEUES"] = str(queues)
    if fused:
        env["ROUNDTABLE_FUSED_AR"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    if r.returncode != 0:
        print(r.stdout[-1500:], r.stderr[-3000:], flush=True)
        raise SystemExit(f"tp{nproc} q{queues} failed rc={r.returncode}")
    return torch.load(out, weights_only=True)


def main():
    ref = run(1)
    cos = torch.nn.functional.cosine_similarity
    for nproc, q in ((4, 4), (4, 2), (8, 2)):
        got = run(nproc, q, fused=True, extra=("--poll-limit", "262144"))
        errs = [e for e in got["errors"] if e is not None]
        row = {"tp": nproc, "queues_per_rank": q, "fused_ar": got["fused_ar"], "fused_ar_calls": got["fused_ar_calls"],
               "graphs": all(got["graphs_per_rank"]), "errors": len(errs), "flag_errors": bool(got["flag_errors"]),
               "ids_equal_tp1": got["ids"] == ref["ids"],
               "decode_cos": round(float(cos(got["decode_logits"][None], ref["decode_logits"][None])), 6)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
