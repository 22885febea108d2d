#!/bin/bash
# round-5 GPU pass C: two-micro-batch probe at tp 8 / 4; driver-config bench A/B of the attention loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05c
export PYTHONUNBUFFERED=1
for t in 8 4; do
  timeout -k 10 300 python -u tools/probes/microbatch_tp8.py --tp $t --ctx 8192 --layers 8 --comm 0,5 \
    > gpurun_out/r05c/microbatch_tp$t.log 2>&1 || { echo "probe tp$t failed"; tail -30 gpurun_out/r05c/microbatch_tp$t.log; exit 1; }
  grep comm_us gpurun_out/r05c/microbatch_tp$t.log
done
for v in 0 d 0 d; do
  if [ $v = 0 ]; then export RT_ATTN_PP=0; else unset RT_ATTN_PP; fi
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r05c/bench_pp$v.json \
    > gpurun_out/r05c/bench_pp$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r05c/bench_pp$v.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05c/bench_pp$v.json')); print('PP=$v', d['value'], d['ms_per_round'], d['config']['seq_len'], d['config']['context_tokens_per_knight_mean'])"
done
