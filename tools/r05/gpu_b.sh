#!/bin/bash
# round-5 GPU pass B: ping-pong attention loop — numerics, then A/B vs the copy loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05b
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "decode or paged" \
  > gpurun_out/r05b/t_attn.log 2>&1 || { echo "attn tests failed"; tail -40 gpurun_out/r05b/t_attn.log; exit 1; }
tail -2 gpurun_out/r05b/t_attn.log
for pp in 0 1 0 1; do
  RT_ATTN_PP=$pp timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --shared 22000:1500,40000:1500 --splits 6,8,10 \
    > gpurun_out/r05b/gattn_tp1_pp$pp.log 2>&1 || { echo "mb tp1 failed"; tail -20 gpurun_out/r05b/gattn_tp1_pp$pp.log; exit 1; }
  echo "== tp1 PP=$pp"; grep "grouped" gpurun_out/r05b/gattn_tp1_pp$pp.log | grep -v "^|"
  RT_ATTN_PP=$pp timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 8,4 --shared 22000:1500 --splits 32,64 \
    > gpurun_out/r05b/gattn_tp8_pp$pp.log 2>&1 || { echo "mb tp8 failed"; tail -20 gpurun_out/r05b/gattn_tp8_pp$pp.log; exit 1; }
  echo "== tp8/4 PP=$pp"; grep "grouped" gpurun_out/r05b/gattn_tp8_pp$pp.log | grep -v "^|"
done
