#!/bin/bash
# round-5 GPU pass BB: prefill key split below 1/2 (current) vs all of the CUs — driver-config
# bench A/B/A/B, compared on engine_prefill_ms_per_round
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05bb
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  for f in 0.5 1.0; do
    ROUNDTABLE_PREFILL_SPLIT_BELOW=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench_f${f}_$pass.json \
      2> $D/bench_f${f}_$pass.err || { tail -20 $D/bench_f${f}_$pass.err; exit 1; }
    python -c "
import json; d = json.loads(open('$D/bench_f${f}_$pass.json').read().strip().splitlines()[-1]); x = d['detail']
print('split below $f pass $pass', d['value'], d['ms_per_step'], 'prefill', x['engine_prefill_ms_per_round'], 'decode', x['engine_decode_ms_per_round'])"
  done
done
