#!/bin/bash
# round-6 GPU pass AD: Llama 3.1 / 3.2 presets end to end — decode kernels at G = 3 (3.2-3B),
# then the table shape (3 knights, shared, parallel rounds, 10 + 3 rounds) on 3.2-1B, 3.2-3B, 3.1-8B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06ad
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "paged_decode and 24-8" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for m in llama3.2-1b llama3.2-3b llama3.1-8b; do
  timeout -k 10 400 python -u bench.py --model $m --steps 10 --warmup 3 > $D/bench_$m.json 2> $D/bench_$m.err \
    || { tail -20 $D/bench_$m.err; exit 1; }
  echo "$m: $(python -c "import json;d=json.load(open('$D/bench_$m.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'], d['config']['seq_len'])")"
done
