#!/bin/bash
# round-6 GPU pass J: driver-config simulated tp records, compute-only and with device-simulated comm
# usage: gpu_g.sh parallel|sequential
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mode=${1:-parallel}
sfx=$([ "$mode" = sequential ] && echo _seq || echo "")
mkdir -p gpurun_out/r06j
export PYTHONUNBUFFERED=1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --round-mode $mode "$@" --out gpurun_out/r06j/$name.json \
    > gpurun_out/r06j/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/r06j/$name.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r06j/$name.json')); print('$name', d['value'], d['ms_per_round'], round(d['detail']['engine_decode_ms_per_round'], 1), d['detail'].get('sim_comm'))"
}
run sim1$sfx --gpus 1
for t in 8 4 2; do
  run sim$t$sfx --simulate-tp $t --sim-k9-us 0 --sim-gather-us 0
  run sim${t}${sfx}_comm5 --simulate-tp $t --sim-k9-us 5 --sim-gather-us 9.5
done
