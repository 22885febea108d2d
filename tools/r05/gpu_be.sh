#!/bin/bash
# round-5 GPU pass BE: last check of the in-tree extension — kernel + engine tests and smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05be
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
