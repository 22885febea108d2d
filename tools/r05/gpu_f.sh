#!/bin/bash
# round-5 GPU pass F: full GPU suite + smoke on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05f
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05f/gpu_tests_full.log 2>&1; rc=$?
tail -5 gpurun_out/r05f/gpu_tests_full.log
grep -E "FAILED|ERROR" gpurun_out/r05f/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05f/smoke.log 2>&1 || { tail -20 gpurun_out/r05f/smoke.log; exit 1; }
tail -2 gpurun_out/r05f/smoke.log
