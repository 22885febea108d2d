#!/bin/bash
# round-5 GPU pass AR: tp 8 shard (1 KV head per rank) grouped attention + combine vs split count
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ar
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 8 --batch 3 --shared 22000:1500,6000:800,40000:1500 \
    --splits 32,40,48,56,64 > $D/tp8_$pass.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 4 --batch 3 --shared 22000:1500,6000:800,40000:1500 \
    --splits 24,32,42,48 > $D/tp4_$pass.log 2>&1 || exit 1
  echo "pass $pass"; grep -h "^| decode attn grouped" $D/tp8_$pass.log $D/tp4_$pass.log
done
