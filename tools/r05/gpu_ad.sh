#!/bin/bash
# round-5 GPU pass AD: fused decode up to 32 rows (two 16-row blocks) — numerics + fixed-batch A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ad
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_serve.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -m gpu > $D/tests.log 2>&1 || { echo "tests failed"; tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for pass in 1 2; do
  for mode in old new; do
    if [ $mode = old ]; then export ROUNDTABLE_FUSED_ROWS=16; else unset ROUNDTABLE_FUSED_ROWS; fi
    for k in 32 24; do
      timeout -k 10 400 python -u bench.py --knights-per-table $k --steps 3 --warmup 1 --new-tokens 256 \
        --out $D/b${k}_${mode}_$pass.json > $D/b${k}_${mode}_$pass.log 2>&1 || { tail -20 $D/b${k}_${mode}_$pass.log; exit 1; }
      python -c "
import json; d=json.load(open('$D/b${k}_${mode}_$pass.json')); dd=d['detail']
print('$mode pass $pass knights $k', d['value'], 'tok/s; decode ms/round', dd['engine_decode_ms_per_round'], 'failed', dd['failed_turns'], 'graphs', dd.get('graphs_per_rank'))"
    done
  done
done
unset ROUNDTABLE_FUSED_ROWS
timeout -k 10 300 python -u tools/serve_bench.py --clients 32 --requests 64 --prompt-words 100 --max-tokens 256 --max-batch 32 \
  > $D/s32_256.log 2>&1 && tail -1 $D/s32_256.log
