#!/bin/bash
# round-6 GPU pass AC: per-kernel HBM bytes of the decode step's kernels (rocprofv3 counters,
# FETCH_SIZE and WRITE_SIZE in separate passes) over the microbench at the driver's shapes
# (Llama-3-8B, 3 rows: the skinny GEMMs; grouped attention 22K shared + 1.5K own keys)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06ac
mkdir -p $D
export PYTHONUNBUFFERED=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $D/pmc_$c -o pmc -- \
    python3 tools/microbench.py --only gemm > $D/pmc_gemm_$c.log 2>&1 || { tail -20 $D/pmc_gemm_$c.log; exit 1; }
  python3 tools/pmc_summary.py $D/pmc_$c $D/gemm_$c.md --counter $c > /dev/null
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $D/pmca_$c -o pmc -- \
    python3 tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 --shared 22000:1500 \
    > $D/pmc_attn_$c.log 2>&1 || { tail -20 $D/pmc_attn_$c.log; exit 1; }
  python3 tools/pmc_summary.py $D/pmca_$c $D/attn_$c.md --counter $c > /dev/null
  echo "== $c"; head -14 $D/gemm_$c.md | cut -c1-230; grep -h "paged_decode\|decode_combine" $D/attn_$c.md | cut -c1-230
  find $D/pmc_$c $D/pmca_$c -name "*.csv" -size +20M -delete
done
