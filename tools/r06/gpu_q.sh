#!/bin/bash
# round-6 GPU pass Q: config 5 shape (2 knights of Llama-3-70B on ONE GPU: one shuffled weight copy,
# the unshuffle prefill path) on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06q
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench.py --model llama3-70b --knights-per-table 2 --steps 2 --warmup 1 \
  > $D/cfg5shape_llama70b_tp1.json 2> $D/cfg5shape.err || { tail -30 $D/cfg5shape.err; exit 1; }
python -c "import json;d=json.load(open('$D/cfg5shape_llama70b_tp1.json'));print(d['value'], d['ms_per_round'], d['detail']['failed_turns'], d['detail'].get('engine_load_s'))"
