#!/bin/bash
# round-6 GPU pass H: counter evidence for the decode attention's K/V stream — L1->L2 read requests
# and HBM (EA) read requests per launch, round-5 tree (row-major K, default-policy loads) vs now
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06h
mkdir -p $D
export PYTHONUNBUFFERED=1
for t in base new; do
  dir=.; [ $t = base ] && dir=ab_base
  timeout -s KILL 240 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-trace --output-format csv -d $D/pmc_$t -o pmc -- \
    python3 $dir/tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 --shared 22000:1500 \
    > $D/pmc_$t.log 2>&1 || { tail -20 $D/pmc_$t.log; exit 1; }
  for c in TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum; do
    python3 tools/pmc_summary.py $D/pmc_$t $D/pmc_${t}_$c.md --counter $c > /dev/null 2>&1 || true
  done
  echo "== $t"; grep -h "paged_decode\|decode_combine" $D/pmc_${t}_*.md | cut -c1-220
  find $D/pmc_$t -name "*.csv" -size +20M -delete
done
