#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05e
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/probes/fused_mlp_tp.py --tp 8,4 --calls 40 > gpurun_out/r05e/fused_mlp_phases.log 2>&1 \
  || { echo "fused mlp probe failed"; tail -30 gpurun_out/r05e/fused_mlp_phases.log; exit 1; }
grep '"tp"' gpurun_out/r05e/fused_mlp_phases.log | grep -v rows
