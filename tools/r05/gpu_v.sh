#!/bin/bash
# round-5 GPU pass V: where tp 1 grouped attention + combine time goes (latency probes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05v
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
for cfg in "probe1 RT_ATTN_PROBE=1" "probe2 RT_ATTN_PROBE=2" "probe3 RT_ATTN_PROBE=3" "nocombine RT_ATTN_SKIP_COMBINE=1" "full X=0"; do
  set -- $cfg
  env $2 timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --shared 6000:800,22000:1500,40000:1500 --splits 8 \
    > $D/$1_$pass.log 2>&1 || { echo "$1 failed"; tail -20 $D/$1_$pass.log; exit 1; }
  echo "$1 pass $pass"; grep "^| decode attn grouped" $D/$1_$pass.log
done
done
