#!/bin/bash
# round-6 GPU pass S: the split combine loads min(B, 16/G) x splits slots per row instead of
# (16/G) x splits (RT_COMBINE_FULL_BOUND=1 = the old bound) — tests, microbench, bench A/B/A/B,
# sequential A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06s
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for fb in 1 0; do
  RT_COMBINE_FULL_BOUND=$fb timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 \
    --shared 22000:1500,40000:1500,6000:800 > $D/g_fb$fb.log 2>&1 || exit 1
  RT_COMBINE_FULL_BOUND=$fb timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 1 --splits 32 \
    --shared 25000:0 > $D/b1_fb$fb.log 2>&1 || exit 1
  echo "FULL_BOUND=$fb"; grep -h "^| decode attn grouped" $D/g_fb$fb.log $D/b1_fb$fb.log
done
for pass in 1 2; do
  for fb in 1 0; do
    RT_COMBINE_FULL_BOUND=$fb timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_fb${fb}_$pass.json \
      2> $D/bench_fb${fb}_$pass.err || { tail -20 $D/bench_fb${fb}_$pass.err; exit 1; }
    echo "fb=$fb pass $pass: $(python -c "import json;d=json.load(open('$D/bench_fb${fb}_$pass.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for fb in 1 0; do
  RT_COMBINE_FULL_BOUND=$fb timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --round-mode sequential \
    > $D/seq_fb$fb.json 2> $D/seq_fb$fb.err || { tail -20 $D/seq_fb$fb.err; exit 1; }
  echo "seq fb=$fb: $(python -c "import json;d=json.load(open('$D/seq_fb$fb.json'));print(d['value'], d['ms_per_step'])")"
done
