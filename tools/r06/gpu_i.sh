#!/bin/bash
# round-6 GPU pass I: which counters this box exposes, then L1 / TA activity of the decode attention
# (round-5 tree vs now)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06i
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -s KILL 120 rocprofv3 --list-avail > $D/counters.txt 2>&1 || true
grep -oE "^\s*(TA|TD|TCP)_[A-Z0-9_]+" $D/counters.txt | sort -u | head -80
for t in base new; do
  dir=.; [ $t = base ] && dir=ab_base
  timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TD_BUSY_avr \
    --kernel-trace --output-format csv -d $D/pmc_$t -o pmc -- \
    python3 $dir/tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 --shared 22000:1500 \
    > $D/pmc_$t.log 2>&1 || { tail -20 $D/pmc_$t.log; exit 1; }
  for c in TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TD_BUSY_avr; do
    python3 tools/pmc_summary.py $D/pmc_$t $D/pmc_${t}_$c.md --counter $c > /dev/null 2>&1 || true
    echo "== $t $c"; grep -h "paged_decode_kernel<128, 16" $D/pmc_${t}_$c.md | head -1 | cut -c1-200
  done
  find $D/pmc_$t -name "*.csv" -size +20M -delete
done
