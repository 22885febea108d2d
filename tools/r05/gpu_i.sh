#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05i
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/probes/sampler_real_logits.py > gpurun_out/r05i/sampler_real.log 2>&1 \
  || { echo "probe failed"; tail -30 gpurun_out/r05i/sampler_real.log; exit 1; }
tail -1 gpurun_out/r05i/sampler_real.log
