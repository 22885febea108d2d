#!/bin/bash
# round-5 GPU pass J: full-depth rehearsal of the driver's N = 2 command on one GPU (2 gloo ranks)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05j
export PYTHONUNBUFFERED=1
ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 20 --warmup 5 --kv-fraction 0.4 \
  --out gpurun_out/r05j/tp2_full_depth.json > gpurun_out/r05j/tp2_full_depth.log 2>&1 \
  || { echo "rehearsal failed"; tail -30 gpurun_out/r05j/tp2_full_depth.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r05j/tp2_full_depth.json')); dd=d['detail']
print(d['value'], d['ms_per_round'], dd['failed_turns'], dd['graph_replays_per_rank'], dd['k9_ll'], dd['k9_us'], dd['k9_resyncs'], dd.get('prediction'))"
