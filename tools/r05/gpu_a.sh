#!/bin/bash
# round-5 GPU pass A: sampler fix, K9 resync, simulated-comm smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05a
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "sample" \
  > gpurun_out/r05a/t_sampler.log 2>&1 || { echo "sampler tests failed"; tail -30 gpurun_out/r05a/t_sampler.log; exit 1; }
tail -3 gpurun_out/r05a/t_sampler.log
timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 400 --timeout-method thread \
  -k "k9_epoch or test_two_rank_tp2_bench" > gpurun_out/r05a/t_dist.log 2>&1 || { echo "dist tests failed"; tail -40 gpurun_out/r05a/t_dist.log; exit 1; }
tail -3 gpurun_out/r05a/t_dist.log
for sk in 0 5; do
  timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 2 --warmup 1 --sim-k9-us $sk \
    --out gpurun_out/r05a/sim8_k9_$sk.json > gpurun_out/r05a/sim8_k9_$sk.log 2>&1 || { echo "sim8 $sk failed"; tail -20 gpurun_out/r05a/sim8_k9_$sk.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05a/sim8_k9_$sk.json')); print('sim8 k9', $sk, d['ms_per_round'], d['detail']['engine_decode_ms_per_round'], d['detail'].get('sim_comm'))"
done
