#!/bin/bash
# round-6 GPU pass L: the final tree through the driver's multi-GPU command shape on ONE card
# (ranks sharing the GPU over gloo + K9 IPC: correctness, not performance) at N = 2 (25 rounds)
# and N = 8 (4 rounds), then the fused-MLP fold's upper bound at tp 1 / tp 2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06l
mkdir -p $D
export PYTHONUNBUFFERED=1
summ() {
  python -c "
import json; d=json.load(open('$1')); dd=d['detail']
print('$2', d['value'], d['ms_per_round'], 'failed', dd['failed_turns'], 'replays', dd['graph_replays_per_rank'], 'graphs', dd['graphs_per_rank'], 'll', dd['k9_ll'], 'k9_us', dd['k9_us'], 'resyncs', dd['k9_resyncs'], 'fallbacks', dd['capture_fallbacks'])"
}
ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 20 --warmup 5 --kv-fraction 0.4 \
  --out $D/tp2_rehearsal.json > $D/tp2_rehearsal.log 2>&1 || { echo "tp2 rehearsal failed"; tail -40 $D/tp2_rehearsal.log; exit 1; }
summ $D/tp2_rehearsal.json tp2
ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 8 --steps 3 --warmup 1 --kv-fraction 0.075 \
  --out $D/tp8_rehearsal.json > $D/tp8_rehearsal.log 2>&1 || { echo "tp8 rehearsal failed"; tail -40 $D/tp8_rehearsal.log; exit 1; }
summ $D/tp8_rehearsal.json tp8
timeout -k 10 400 python -u tools/probes/fused_mlp_tp.py --tp 1,2 > $D/fused_mlp_tp1.log 2>&1 || { tail -20 $D/fused_mlp_tp1.log; exit 1; }
grep '^{"tp"' $D/fused_mlp_tp1.log
