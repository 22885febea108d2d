#!/bin/bash
# round-5 GPU pass U: EPI_AR correct at tp 4 / 8 with per-rank CU slices; shared-GPU TP tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05u
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "cu_split or tp_fused_decode or strong_scaling_bench or contained" > $D/tests.log 2>&1; rc=$?
tail -15 $D/tests.log
exit $rc
