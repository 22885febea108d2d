#!/bin/bash
# round-5 GPU pass D: fused-MLP launch folding A/B at shard shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05d
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/probes/fused_mlp_tp.py --tp 8,4,2 --calls 40 > gpurun_out/r05d/fused_mlp.log 2>&1 \
  || { echo "fused mlp probe failed"; tail -30 gpurun_out/r05d/fused_mlp.log; exit 1; }
grep '"tp"' gpurun_out/r05d/fused_mlp.log | grep -v rows
timeout -k 10 400 python -u tools/probes/fused_mlp_tp.py --tp 8,4 --calls 40 > gpurun_out/r05d/fused_mlp_2.log 2>&1 \
  || { echo "fused mlp probe 2 failed"; tail -30 gpurun_out/r05d/fused_mlp_2.log; exit 1; }
grep '"tp"' gpurun_out/r05d/fused_mlp_2.log | grep -v rows
