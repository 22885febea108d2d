#!/bin/bash
# round-5 GPU pass X: multi-tile skinny GEMM for serving batches (M > 4): numerics, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05x
mkdir -p $D
export PYTHONUNBUFFERED=1
for tn in 2 4; do
  RT_SKINNY_TN=$tn timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $D/tests_tn$tn.log 2>&1 || { echo "tests TN=$tn failed"; tail -30 $D/tests_tn$tn.log; exit 1; }
  echo "TN=$tn: $(tail -1 $D/tests_tn$tn.log)"
done
for b in 16 8; do
  for cfg in "0 402" "2 402" "2 802" "4 402" "4 802"; do
    set -- $cfg
    RT_SKINNY_TN=$1 RT_SKINNY_TNCFG=${2:0:1}x${2:2:1} timeout -k 10 300 python -u tools/microbench.py --only gemm --batch $b \
      > $D/mb_b${b}_tn$1_$2.log 2>&1 || { echo "mb failed"; tail -20 $D/mb_b${b}_tn$1_$2.log; exit 1; }
    echo "batch $b TN=$1 cfg=$2"; grep "^| skinny" $D/mb_b${b}_tn$1_$2.log | grep -v "plain, unpaired\|gate_up-plain"
  done
done
