#!/bin/bash
# round-6 GPU pass B: chunk-major K cache + nontemporal K/V loads — kernel / GEMM / engine tests,
# smoke, attention microbench (nt on/off), then the driver-config bench A/B/A/B against the
# round-5 tree (ab_base/, built from HEAD before the change)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06b
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
for lm in 0 1; do
  RT_ATTN_LM=$lm timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 \
    --shared 22000:1500,40000:1500,6000:800 > $D/tp1_lm${lm}.log 2>&1 || exit 1
  RT_ATTN_LM=$lm timeout -k 10 300 python -u tools/microbench.py --only attn --batch 1 --ctx 25000 --splits 32 \
    > $D/b1_lm${lm}.log 2>&1 || exit 1
  echo "LM=$lm"; grep -h "^| decode attn" $D/tp1_lm${lm}.log $D/b1_lm${lm}.log | grep -v "ctx=1500"
done
for pass in 1 2; do
  timeout -k 10 400 python -u ab_base/bench.py --steps 20 --warmup 5 > $D/bench_base_$pass.json 2> $D/bench_base_$pass.err || { tail -20 $D/bench_base_$pass.err; exit 1; }
  echo "base $pass: $(python -c "import json;d=json.load(open('$D/bench_base_$pass.json'));print(d['value'], d['ms_per_step'])")"
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_new_$pass.json 2> $D/bench_new_$pass.err || { tail -20 $D/bench_new_$pass.err; exit 1; }
  echo "new  $pass: $(python -c "import json;d=json.load(open('$D/bench_new_$pass.json'));print(d['value'], d['ms_per_step'])")"
done
