#!/bin/bash
# round-5 GPU pass Z: multi-tile GEMM with the K-split for o / down (M > 4): numerics + microbench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05z
mkdir -p $D
export PYTHONUNBUFFERED=1
: timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_serve.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -m gpu > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for pass in 1 2; do
  for tns in 0 1; do
    RT_SKINNY_TNS=$tns timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 16 > $D/mb_b16_tns${tns}_$pass.log 2>&1 || exit 1
    echo "M=16 TNS=$tns pass $pass"; grep "^| skinny o \|^| skinny down" $D/mb_b16_tns${tns}_$pass.log
    RT_SKINNY_TNS=$tns timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 8 > $D/mb_b8_tns${tns}_$pass.log 2>&1 || exit 1
    echo "M=8 TNS=$tns pass $pass"; grep "^| skinny o \|^| skinny down" $D/mb_b8_tns${tns}_$pass.log
  done
done
