#!/bin/bash
# round-5 GPU pass AQ: split-combine lane count at 10 splits (40 slots per row)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05aq
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  for nsl in 32 40 48 16; do
    RT_COMBINE_NSL=$nsl timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --shared 22000:1500,6000:800,40000:1500 \
      --splits 10 > $D/nsl${nsl}_$pass.log 2>&1 || exit 1
    echo "NSL=$nsl pass $pass"; grep "^| decode attn grouped" $D/nsl${nsl}_$pass.log
  done
done
