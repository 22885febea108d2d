#!/bin/bash
# round-6 GPU pass K: the fused-MLP fold's upper bound at tp 1 (whole Llama-3-8B MLP, M = 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06k
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/probes/fused_mlp_tp.py --tp 1,2 > $D/fused_mlp_tp1.log 2>&1 || { tail -20 $D/fused_mlp_tp1.log; exit 1; }
grep '^{"tp"' $D/fused_mlp_tp1.log
