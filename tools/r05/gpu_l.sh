#!/bin/bash
# round-5 GPU pass L: the driver's N = 4 and N = 8 bench commands rehearsed on ONE GPU (gloo ranks
# sharing the card, K9 over IPC), fewer rounds; stage transitions logged per rank
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05l
export PYTHONUNBUFFERED=1
for N in 4 8; do
  frac=$(python -c "print(round(0.6 / $N, 3))")
  ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 540 python -u bench.py --gpus $N --steps 3 --warmup 1 --kv-fraction $frac \
    --out gpurun_out/r05l/tp${N}_rehearsal.json > gpurun_out/r05l/tp${N}_rehearsal.log 2>&1 \
    || { echo "tp$N rehearsal failed"; tail -40 gpurun_out/r05l/tp${N}_rehearsal.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r05l/tp${N}_rehearsal.json')); dd=d['detail']
print($N, d['value'], d['ms_per_round'], dd['failed_turns'], dd['graph_replays_per_rank'], dd['graphs_per_rank'], dd['k9_ll'], dd['k9_us'], dd['k9_gather'], dd['k9_resyncs'], dd['capture_fallbacks'])"
done
