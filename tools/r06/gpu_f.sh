#!/bin/bash
# round-6 GPU pass F: serve load re-measured with zero losses: the batch
# default (16 vs 32 rows), 64 clients (max batch 32 vs 64), and the round-5 K-read-order claim on
# the round-5 tree (ab_base/, its serve.py replaced by the fixed one: 1024-deep listen backlog)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06f
mkdir -p $D
export PYTHONUNBUFFERED=1
sb() {  # name, dir, env..., -- args
  local name=$1 dir=$2; shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 400 python -u $dir/tools/serve_bench.py "$@" > $D/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep '^{' $D/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['scheduler']; print(d['value'], 'tok/s', d['completed_requests'], 'done', d['failed_requests'], 'failed, rows/step', round(s['decode_rows']/max(1,s['decode_steps']),1), 'p50/p99', d['latency_s_p50'], d['latency_s_p99'])")"
  [ $rc -le 1 ]
}
for pass in 1 2; do
  for mb in 16 32; do
    sb c32_mb${mb}_$pass . X=0 -- --clients 32 --requests 96 --prompt-words 100 --max-tokens 256 --max-batch $mb || exit 1
  done
  for mb in 32 64; do
    sb c64_mb${mb}_$pass . X=0 -- --clients 64 --requests 192 --prompt-words 100 --max-tokens 256 --max-batch $mb || exit 1
  done
  for kp in 0 1; do
    sb base_kperm${kp}_$pass ab_base RT_ATTN_KPERM=$kp -- --clients 32 --requests 96 --prompt-words 100 --max-tokens 256 --max-batch 16 || exit 1
  done
done
