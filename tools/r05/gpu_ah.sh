#!/bin/bash
# round-5 GPU pass AH: same-box A/B/A/B of the driver-config bench, tree before the serving-batch
# GEMM work (ab_old/, commit aa3a3a0) vs the current tree — is the 3-row headline path unchanged?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ah
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  for t in old new; do
    if [ $t = old ]; then B=ab_old/bench.py; else B=bench.py; fi
    timeout -k 10 400 python -u $B --steps 20 --warmup 5 --out $D/bench_${t}_$pass.json > $D/bench_${t}_$pass.log 2>&1 || { tail -20 $D/bench_${t}_$pass.log; exit 1; }
    python -c "import json; d=json.load(open('$D/bench_${t}_$pass.json')); print('$t pass $pass', d['value'], d['ms_per_round'], d['detail']['engine_decode_ms_per_round'], d['detail']['failed_turns'])"
  done
done
