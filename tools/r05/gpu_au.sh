#!/bin/bash
# odd tile counts on the serving-batch GEMM launches, then the whole GPU suite and smoke()
set -o pipefail
mkdir -p gpurun_out/r05au
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k odd_tile -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r05au/odd_tile.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r05au/gpu_tests_full.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05au/smoke.log 2>&1
