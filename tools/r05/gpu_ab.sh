#!/bin/bash
# round-5 GPU pass AB: decode at a fixed batch of 16 / 8 rows (bench.py with a 16- / 8-knight table,
# private prompts): one-tile GEMMs vs the serving-batch multi-tile rule, A/B/A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ab
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  for mode in old new; do
    if [ $mode = old ]; then export RT_SKINNY_TN=1 RT_SKINNY_TNS=0; else unset RT_SKINNY_TN RT_SKINNY_TNS; fi
    for k in 16 8; do
      timeout -k 10 400 python -u bench.py --knights-per-table $k --steps 3 --warmup 1 --new-tokens 256 \
        --out $D/b${k}_${mode}_$pass.json > $D/b${k}_${mode}_$pass.log 2>&1 || { tail -20 $D/b${k}_${mode}_$pass.log; exit 1; }
      python -c "
import json; d=json.load(open('$D/b${k}_${mode}_$pass.json')); dd=d['detail']
print('$mode pass $pass knights $k', d['value'], 'tok/s; decode ms/round', dd['engine_decode_ms_per_round'], 'failed', dd['failed_turns'])"
    done
  done
done
