#!/bin/bash
# round-5 GPU pass AE: 32-row GEMMs (lm_head 4 tiles x 2 row blocks), numerics + rows sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ae
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "serving or rope_epilogue or fused_decode" > $D/tests.log 2>&1 || { echo "tests failed"; tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for b in 32 24 16; do
  timeout -k 10 300 python -u tools/microbench.py --only gemm --batch $b > $D/mb_b$b.log 2>&1 || exit 1
  echo "M=$b"; grep "^| skinny" $D/mb_b$b.log | grep -v "gate_up-plain\|balanced"
done
for pass in 1 2; do
  for k in 32 24; do
    timeout -k 10 400 python -u bench.py --knights-per-table $k --steps 3 --warmup 1 --new-tokens 256 \
      --out $D/b${k}_$pass.json > $D/b${k}_$pass.log 2>&1 || { tail -20 $D/b${k}_$pass.log; exit 1; }
    python -c "
import json; d=json.load(open('$D/b${k}_$pass.json')); dd=d['detail']
print('pass $pass knights $k', d['value'], 'tok/s; decode ms/round', dd['engine_decode_ms_per_round'], 'failed', dd['failed_turns'])"
  done
done
