#!/bin/bash
# round-5 GPU pass AM: grouped attention split count at tensor-parallel shard shapes (B = 3):
# 3/4 of the CUs (current) vs the whole chip
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05am
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 2 --batch 3 --shared 22000:1500,6000:800,40000:1500 --splits 16,21 \
    > $D/tp2_$pass.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 4 --batch 3 --shared 22000:1500,6000:800,40000:1500 --splits 32,42 \
    > $D/tp4_$pass.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --shared 22000:1500,6000:800,40000:1500 --splits 8,10 \
    > $D/tp1_$pass.log 2>&1 || exit 1
  echo "pass $pass"; grep -h "^| decode attn grouped" $D/tp2_$pass.log $D/tp4_$pass.log $D/tp1_$pass.log
done
