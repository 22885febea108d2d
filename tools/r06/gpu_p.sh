#!/bin/bash
# round-6 GPU pass P: the experiment extension's own GPU tests (persistent layer, combine-in-o,
# LDS-ring GEMM) on the chunk-major K layout
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06p
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tools/experiments -m gpu -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $D/exp_tests.log 2>&1; rc=$?
tail -3 $D/exp_tests.log; grep -E "FAILED|ERROR" $D/exp_tests.log | head
exit $rc
