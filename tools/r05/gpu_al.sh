#!/bin/bash
# round-5 GPU pass AL: o / down at 9-16 rows — 2 tiles x 2 K halves vs 4 tiles x 4 K quarters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05al
mkdir -p $D
export PYTHONUNBUFFERED=1
RT_SKINNY_TNS=4 timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "serving" > $D/tests_tns4.log 2>&1 || { tail -30 $D/tests_tns4.log; exit 1; }
tail -1 $D/tests_tns4.log
for pass in 1 2; do
  for tns in 1 4; do
    RT_SKINNY_TNS=$tns timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 16 > $D/mb_tns${tns}_$pass.log 2>&1 || exit 1
    echo "TNS=$tns pass $pass"; grep "split ws" $D/mb_tns${tns}_$pass.log
  done
done
