#!/bin/bash
# round-6 GPU pass AE: 32x32 prefill for GQA groups that are not powers of two (padded head slots:
# Qwen2.5 G = 7 in 8, Llama-3.2-3B G = 3 in 4) — prefill tests (whole tiles and key split) against
# the fp32 oracle, then Qwen2.5-7B / Llama-3.2-3B at the table shape, 32x32 vs the 16x16 kernel
# (ROUNDTABLE_PREFILL16=1, the previous path for these groups), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06ae
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_hf_parity.py -x -q -m gpu -k "prefill or transformers" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for m in qwen2.5-7b llama3.2-3b; do
  for p16 in 1 0; do
    if [ $p16 = 1 ]; then export ROUNDTABLE_PREFILL16=1; else unset ROUNDTABLE_PREFILL16; fi
    timeout -k 10 400 python -u bench.py --model $m --steps 10 --warmup 3 > $D/bench_${m}_p16$p16.json \
      2> $D/bench_${m}_p16$p16.err || { tail -20 $D/bench_${m}_p16$p16.err; exit 1; }
    echo "$m prefill16=$p16: $(python -c "import json;d=json.load(open('$D/bench_${m}_p16$p16.json'));x=d['detail'];print(d['value'], d['ms_per_step'], x['failed_turns'], x['engine_prefill_ms_per_round'])")"
  done
done
