#!/bin/bash
# round-6 GPU pass U: decode attention with K/V staged through LDS by LDS-DMA (RT_ATTN_LM=7,
# attn_core.h LM_GLDS) vs the register-staged default (RT_ATTN_LM=3) — numerics against the fp32
# oracle with the staged form forced, microbench on one box, driver-config bench A/B/A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06u
mkdir -p $D
export PYTHONUNBUFFERED=1
RT_ATTN_LM=7 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "paged_decode" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests_lm7.log 2>&1 || { tail -40 $D/tests_lm7.log; exit 1; }
tail -1 $D/tests_lm7.log
for pass in 1 2; do
  for lm in 3 7; do
    RT_ATTN_LM=$lm timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 \
      --shared 22000:1500,40000:1500,6000:800 > $D/g_lm${lm}_$pass.log 2>&1 || { tail -20 $D/g_lm${lm}_$pass.log; exit 1; }
    RT_ATTN_LM=$lm timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 1 --splits 32 \
      --shared 25000:0 > $D/b1_lm${lm}_$pass.log 2>&1 || { tail -20 $D/b1_lm${lm}_$pass.log; exit 1; }
    echo "LM=$lm pass $pass"; grep -h "^| decode attn grouped" $D/g_lm${lm}_$pass.log $D/b1_lm${lm}_$pass.log
  done
done
for pass in 1 2; do
  for lm in 3 7; do
    RT_ATTN_LM=$lm timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_lm${lm}_$pass.json \
      2> $D/bench_lm${lm}_$pass.err || { tail -20 $D/bench_lm${lm}_$pass.err; exit 1; }
    echo "lm=$lm pass $pass: $(python -c "import json;d=json.load(open('$D/bench_lm${lm}_$pass.json'));print(d['value'], d['ms_per_step'])")"
  done
done
