#!/bin/bash
# round-5 GPU pass AK: grouped attention on the whole chip from 5 rows — fixed-batch A/B/A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ak
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  for mode in old new; do
    if [ $mode = old ]; then export ROUNDTABLE_GROUPED_FULL_FROM=99; else unset ROUNDTABLE_GROUPED_FULL_FROM; fi
    for k in 16 8; do
      if [ $k = 8 ]; then extra="--model mistral-7b --knights-per-gpu 8 --steps 4 --warmup 1"; else extra="--steps 3 --warmup 1 --new-tokens 256"; fi
      timeout -k 10 400 python -u bench.py --knights-per-table $k $extra --out $D/b${k}_${mode}_$pass.json > $D/b${k}_${mode}_$pass.log 2>&1 \
        || { tail -20 $D/b${k}_${mode}_$pass.log; exit 1; }
      python -c "
import json; d=json.load(open('$D/b${k}_${mode}_$pass.json')); dd=d['detail']
print('$mode pass $pass knights $k', d['value'], 'tok/s; decode ms/round', dd['engine_decode_ms_per_round'], 'failed', dd['failed_turns'])"
    done
  done
done
unset ROUNDTABLE_GROUPED_FULL_FROM
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider -m gpu > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
