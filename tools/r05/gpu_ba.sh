#!/bin/bash
# round-5 GPU pass BA: prefill attention with lane-contiguous K/V chunk loads — kernel tests, then
# microbench A/B/A/B against the previous loads (ab_old/: HEAD before the change, built side by side)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ba
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "prefill" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
P="4096:0,1536:22000,1536:40000,512:22000"
for pass in 1 2; do
  for t in old new; do
    if [ $t = old ]; then M=ab_old/tools/microbench.py; else M=tools/microbench.py; fi
    timeout -k 10 300 python -u $M --only prefill --prefill $P > $D/${t}_$pass.log 2>&1 || { tail -20 $D/${t}_$pass.log; exit 1; }
    echo "$t pass $pass"; grep -h "^| prefill" $D/${t}_$pass.log
  done
done
