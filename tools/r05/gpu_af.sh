#!/bin/bash
# round-5 GPU pass AF: BASELINE configs 3 / 4 / 5-shape on the late round-5 tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05af
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --model mistral-7b --knights-per-table 8 --knights-per-gpu 8 --steps 4 --warmup 1 \
  --out $D/cfg3_mistral7b_8knights.json > $D/cfg3.log 2>&1 || { tail -20 $D/cfg3.log; exit 1; }
python -c "import json; d=json.load(open('$D/cfg3_mistral7b_8knights.json')); print('cfg3', d['value'], d['ms_per_round'], d['detail']['failed_turns'])"
timeout -k 10 500 python -u tools/run_configs.py --config 4 > $D/cfg4.log 2>&1 || { tail -20 $D/cfg4.log; exit 1; }
tail -1 $D/cfg4.log
timeout -k 10 700 python -u bench.py --model llama3-70b --knights-per-table 2 --steps 2 --warmup 1 \
  --out $D/cfg5shape_llama70b_tp1.json > $D/cfg5.log 2>&1 || { tail -20 $D/cfg5.log; exit 1; }
python -c "import json; d=json.load(open('$D/cfg5shape_llama70b_tp1.json')); print('cfg5 shape', d['value'], d['ms_per_round'], d['detail']['failed_turns'])"
