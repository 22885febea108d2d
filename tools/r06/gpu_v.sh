#!/bin/bash
# round-6 GPU pass V: Qwen2 family (q/k/v bias in the fused qkv RoPE epilogue) — bias kernel tests
# on every launch form, HF transformers parity on the HIP path, the driver-config bench A/B against
# the previous build (ab_prev/: the epilogue gained a null-bias branch), Qwen2.5-7B / 0.5B benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06v
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_hf_parity.py -x -v -m gpu -k "rope or transformers" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for t in prev new; do
  if [ $t = prev ]; then R=ab_prev; else R=.; fi
  (cd $R && timeout -k 10 300 python -u tools/microbench.py --only gemm) > $D/gemm_$t.log 2>&1 || { tail -20 $D/gemm_$t.log; exit 1; }
  echo "== gemm $t"; grep -h "skinny qkv" $D/gemm_$t.log
done
for pass in 1 2; do
  for t in prev new; do
    if [ $t = prev ]; then R=ab_prev; else R=.; fi
    (cd $R && timeout -k 10 400 python -u bench.py --steps 20 --warmup 5) > $D/bench_${t}_$pass.json \
      2> $D/bench_${t}_$pass.err || { tail -20 $D/bench_${t}_$pass.err; exit 1; }
    echo "$t pass $pass: $(python -c "import json;d=json.load(open('$D/bench_${t}_$pass.json'));print(d['value'], d['ms_per_step'])")"
  done
done
timeout -k 10 400 python -u bench.py --model qwen2.5-7b --steps 20 --warmup 5 > $D/bench_qwen7b.json \
  2> $D/bench_qwen7b.err || { tail -20 $D/bench_qwen7b.err; exit 1; }
echo "qwen2.5-7b: $(python -c "import json;d=json.load(open('$D/bench_qwen7b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
timeout -k 10 400 python -u bench.py --model qwen2.5-0.5b --steps 10 --warmup 3 > $D/bench_qwen05b.json \
  2> $D/bench_qwen05b.err || { tail -20 $D/bench_qwen05b.err; exit 1; }
echo "qwen2.5-0.5b: $(python -c "import json;d=json.load(open('$D/bench_qwen05b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
