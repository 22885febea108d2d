#!/bin/bash
# round-6 GPU pass T: GEMM kernarg prologue in one scalar batch (tile_base branch-free, so the load
# of N is no longer sunk into the k-chunked branch) — GEMM / kernel tests, GEMM microbench and
# driver-config bench A/B/A/B against the previous commit (ab_prev/)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06t
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for t in prev new; do
  if [ $t = prev ]; then R=ab_prev; else R=.; fi
  (cd $R && timeout -k 10 300 python -u tools/microbench.py --only gemm) > $D/gemm_$t.log 2>&1 || { tail -20 $D/gemm_$t.log; exit 1; }
  echo "== gemm $t"; grep -h "^|" $D/gemm_$t.log | head -30
done
for pass in 1 2; do
  for t in prev new; do
    if [ $t = prev ]; then R=ab_prev; else R=.; fi
    (cd $R && timeout -k 10 400 python -u bench.py --steps 20 --warmup 5) > $D/bench_${t}_$pass.json \
      2> $D/bench_${t}_$pass.err || { tail -20 $D/bench_${t}_$pass.err; exit 1; }
    echo "$t pass $pass: $(python -c "import json;d=json.load(open('$D/bench_${t}_$pass.json'));print(d['value'], d['ms_per_step'])")"
  done
done
