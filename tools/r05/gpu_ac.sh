#!/bin/bash
# round-5 GPU pass AC: would the multi-tile launches help the 3-row headline GEMMs too?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ac
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  for cfg in "5 -1 1" "1 -1 2" "1 2 0" "1 4 0"; do
    set -- $cfg
    if [ "$2" = "-1" ]; then unset RT_SKINNY_TN; else export RT_SKINNY_TN=$2; fi
    RT_SKINNY_TN_MINM=$1 RT_SKINNY_TNS=$3 timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 3 \
      > $D/mb_m$1_tn$2_s$3_$pass.log 2>&1 || { tail -20 $D/mb_m$1_tn$2_s$3_$pass.log; exit 1; }
    echo "minM=$1 TN=$2 TNS=$3 pass $pass"; grep "^| skinny" $D/mb_m$1_tn$2_s$3_$pass.log | grep -v "gate_up-plain"
  done
done
