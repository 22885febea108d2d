#!/bin/bash
# round-5 GPU pass M: the N = 8 rehearsal again with 2 hardware queues per process (8 ranks x 4
# default queues oversubscribe the card's mapped user queues: a K9 call whose peers' queues are not
# mapped waits out its poll bound) and a ~4 s K9 poll bound so any stuck call fails its turn fast
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05m
export PYTHONUNBUFFERED=1
N=8
GPU_MAX_HW_QUEUES=2 ROUNDTABLE_K9_POLL_LIMIT=4194304 ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 600 \
  python -u bench.py --gpus $N --steps 3 --warmup 1 --kv-fraction 0.075 \
  --out gpurun_out/r05m/tp${N}_rehearsal.json > gpurun_out/r05m/tp${N}_rehearsal.log 2>&1 \
  || { echo "tp$N rehearsal failed"; tail -40 gpurun_out/r05m/tp${N}_rehearsal.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r05m/tp${N}_rehearsal.json')); dd=d['detail']
print($N, d['value'], d['ms_per_round'], dd['failed_turns'], dd['graph_replays_per_rank'], dd['graphs_per_rank'], dd['k9_ll'], dd['k9_us'], dd['k9_gather'], dd['k9_resyncs'], dd['capture_fallbacks'])"
