#!/bin/bash
# round-5 GPU pass AA: serving-batch GEMMs final rule — numerics, serving A/B/A/B, headline bench unchanged
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05aa
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_serve.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -m gpu > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for pass in 1 2; do
  for mode in old new; do
    if [ $mode = old ]; then export RT_SKINNY_TN=1 RT_SKINNY_TNS=0; else unset RT_SKINNY_TN RT_SKINNY_TNS; fi
    timeout -k 10 300 python -u tools/serve_bench.py --clients 16 --requests 16 --prompt-words 100 --max-tokens 512 --max-batch 16 \
      > $D/s16_512_${mode}_$pass.log 2>&1 || { tail -20 $D/s16_512_${mode}_$pass.log; exit 1; }
    timeout -k 10 300 python -u tools/serve_bench.py --clients 32 --requests 64 --prompt-words 100 --max-tokens 256 --max-batch 32 \
      > $D/s32_256_${mode}_$pass.log 2>&1 || { tail -20 $D/s32_256_${mode}_$pass.log; exit 1; }
    python -c "
import json
for f in ['$D/s16_512_${mode}_$pass.log', '$D/s32_256_${mode}_$pass.log']:
    d = json.loads(open(f).read().strip().splitlines()[-1]); s = d['scheduler']
    print('$mode pass $pass', f.split('/')[-1], d['value'], 'tok/s rows/step %.1f' % (s['decode_rows'] / s['decode_steps']))"
  done
done
unset RT_SKINNY_TN RT_SKINNY_TNS
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --out $D/bench1.json > $D/bench1.log 2>&1 || { tail -20 $D/bench1.log; exit 1; }
python -c "import json; d=json.load(open('$D/bench1.json')); print('bench', d['value'], d['ms_per_round'], d['detail']['failed_turns'])"
