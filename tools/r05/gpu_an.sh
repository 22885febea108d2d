#!/bin/bash
# round-5 GPU pass AN: driver-config bench, grouped attention on 3/4 of the CUs (8 splits) vs the
# whole chip (10 splits), same box, A/B/A/B/A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05an
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2 3; do
  for f in 0.75 1.0; do
    ROUNDTABLE_GROUPED_CU_FRACTION=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --out $D/bench_f${f}_$pass.json \
      > $D/bench_f${f}_$pass.log 2>&1 || { tail -20 $D/bench_f${f}_$pass.log; exit 1; }
    python -c "import json; d=json.load(open('$D/bench_f${f}_$pass.json')); print('frac $f pass $pass', d['value'], d['ms_per_round'], d['detail']['engine_decode_ms_per_round'])"
  done
done
