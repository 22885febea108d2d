#!/bin/bash
# round-5 GPU pass N: the N = 8 rehearsal in the box's default environment (which exports
# GPU_MAX_HW_QUEUES=4): bench.py's launcher now lowers it to 2 for 8 ranks sharing the card
# (parallel/cluster.py limit_shared_gpu_queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05n
export PYTHONUNBUFFERED=1
echo "box env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
N=8
ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 600 \
  python -u bench.py --gpus $N --steps 3 --warmup 1 --kv-fraction 0.075 \
  --out gpurun_out/r05n/tp${N}_rehearsal.json > gpurun_out/r05n/tp${N}_rehearsal.log 2>&1 \
  || { echo "tp$N rehearsal failed"; tail -40 gpurun_out/r05n/tp${N}_rehearsal.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r05n/tp${N}_rehearsal.json')); dd=d['detail']
print($N, d['value'], d['ms_per_round'], dd['failed_turns'], dd['graph_replays_per_rank'], dd['graphs_per_rank'], dd['k9_ll'], dd['k9_us'], dd['k9_gather'], dd['k9_resyncs'], dd['capture_fallbacks'])"
