#!/bin/bash
# round-6 GPU pass W: Qwen2 family end to end — decode / grouped decode / prefill kernels at
# non-power-of-two GQA groups (G = 7, 3, 12) against the fp32 oracle, HF transformers parity on
# the HIP path, then the driver config on Qwen2.5-7B and Qwen2.5-0.5B (random init)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06w
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_hf_parity.py tests/test_gemm_gpu.py -x -q -m gpu \
  -k "paged_decode or prefill or transformers or rope" --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 400 python -u bench.py --model qwen2.5-7b --steps 20 --warmup 5 > $D/bench_qwen7b.json \
  2> $D/bench_qwen7b.err || { tail -20 $D/bench_qwen7b.err; exit 1; }
echo "qwen2.5-7b: $(python -c "import json;d=json.load(open('$D/bench_qwen7b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
timeout -k 10 400 python -u bench.py --model qwen2.5-0.5b --steps 10 --warmup 3 > $D/bench_qwen05b.json \
  2> $D/bench_qwen05b.err || { tail -20 $D/bench_qwen05b.err; exit 1; }
echo "qwen2.5-0.5b: $(python -c "import json;d=json.load(open('$D/bench_qwen05b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
