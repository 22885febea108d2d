#!/bin/bash
# round-6 GPU pass AG: the driver's N = 2 and N = 8 bench commands rehearsed on ONE card with the
# final tree (ranks share the GPU; gloo control plane; KV pool fraction per rank)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06ag
mkdir -p $D
export PYTHONUNBUFFERED=1
summ() { python3 -c "import json;d=json.load(open('$1'));x=d.get('detail',{});print('$2', d.get('value'), d.get('ms_per_step'), x.get('failed_turns'), d['config'].get('parallelism'), d.get('error'))"; }
ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 5 --warmup 2 --kv-fraction 0.4 \
  --out $D/tp2_rehearsal.json > $D/tp2_rehearsal.log 2>&1 || { echo "tp2 rehearsal failed"; tail -40 $D/tp2_rehearsal.log; exit 1; }
summ $D/tp2_rehearsal.json tp2
ROUNDTABLE_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 8 --steps 3 --warmup 1 --kv-fraction 0.075 \
  --out $D/tp8_rehearsal.json > $D/tp8_rehearsal.log 2>&1 || { echo "tp8 rehearsal failed"; tail -40 $D/tp8_rehearsal.log; exit 1; }
summ $D/tp8_rehearsal.json tp8
