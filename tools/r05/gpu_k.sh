#!/bin/bash
# round-5 GPU pass K: driver-config A/B of the grouped attention's CU share (8 vs 10 splits), new GPU test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05k
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k simulated_tp \
  > gpurun_out/r05k/t_sim.log 2>&1 || { echo "sim test failed"; tail -30 gpurun_out/r05k/t_sim.log; exit 1; }
tail -1 gpurun_out/r05k/t_sim.log
for f in 0.75 0.9375 0.75 0.9375; do
  ROUNDTABLE_GROUPED_CU_FRACTION=$f timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r05k/bench_$f.json \
    > gpurun_out/r05k/bench_$f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r05k/bench_$f.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05k/bench_$f.json')); print('frac $f', d['value'], d['ms_per_round'])"
done
