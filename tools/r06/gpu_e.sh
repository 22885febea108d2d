#!/bin/bash
# round-6 GPU pass E: per-step attention work plan (ops.attn_plan) — decode / engine GPU tests,
# microbench plan on/off, driver-config bench A/B/A/B (ROUNDTABLE_ATTN_PLAN=0 vs 1, same tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06e
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for pl in 0 1; do
  ROUNDTABLE_ATTN_PLAN=$pl timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 \
    --shared 22000:1500,40000:1500,6000:800 > $D/g_plan$pl.log 2>&1 || exit 1
  ROUNDTABLE_ATTN_PLAN=$pl timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 8 --batch 3 --splits 64 \
    --shared 22000:1500 > $D/tp8_plan$pl.log 2>&1 || exit 1
  ROUNDTABLE_ATTN_PLAN=$pl timeout -k 10 300 python -u tools/microbench.py --only attn --batch 1 --ctx 25000 --splits 32 \
    > $D/b1_plan$pl.log 2>&1 || exit 1
  echo "PLAN=$pl"; grep -h "^| decode attn" $D/g_plan$pl.log $D/tp8_plan$pl.log $D/b1_plan$pl.log | grep -v "ctx=1500\|private"
done
for pass in 1 2; do
  for pl in 0 1; do
    ROUNDTABLE_ATTN_PLAN=$pl timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_plan${pl}_$pass.json \
      2> $D/bench_plan${pl}_$pass.err || { tail -20 $D/bench_plan${pl}_$pass.err; exit 1; }
    echo "plan=$pl pass $pass: $(python -c "import json;d=json.load(open('$D/bench_plan${pl}_$pass.json'));print(d['value'], d['ms_per_step'])")"
  done
done
