#!/bin/bash
# round-5 GPU pass AJ: grouped decode attention split count at larger tables (B = 8 / 16 knights)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05aj
mkdir -p $D
export PYTHONUNBUFFERED=1
for b in 16 8 12; do
  timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch $b --shared 11000:300,6000:800,22000:1500 --splits 1,2,3,4 \
    > $D/gattn_b$b.log 2>&1 || { tail -20 $D/gattn_b$b.log; exit 1; }
  echo "B=$b"; grep "^| decode attn grouped" $D/gattn_b$b.log
done
