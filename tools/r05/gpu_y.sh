#!/bin/bash
# round-5 GPU pass Y: multi-tile GEMM default rule — numerics (GEMM, engine, serve tests), the
# serving load test before/after (RT_SKINNY_TN=1 = the old path), and the M = 16 / 3 GEMM rows
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05y
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_serve.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider -m gpu > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for pass in 1 2; do
  for tn in 1 auto; do
    if [ $tn = auto ]; then unset RT_SKINNY_TN; else export RT_SKINNY_TN=$tn; fi
    timeout -k 10 300 python -u tools/serve_bench.py --clients 16 --requests 32 --prompt-words 400 --max-tokens 256 --max-batch 16 \
      > $D/s16_256_tn${tn}_$pass.log 2>&1 || { tail -20 $D/s16_256_tn${tn}_$pass.log; exit 1; }
    timeout -k 10 300 python -u tools/serve_bench.py --clients 16 --requests 16 --prompt-words 100 --max-tokens 512 --max-batch 16 \
      > $D/s16_512_tn${tn}_$pass.log 2>&1 || { tail -20 $D/s16_512_tn${tn}_$pass.log; exit 1; }
    python -c "
import json
for f in ['$D/s16_256_tn${tn}_$pass.log', '$D/s16_512_tn${tn}_$pass.log']:
    d = json.loads(open(f).read().strip().splitlines()[-1]); s = d['scheduler']
    print('TN=$tn pass $pass', f.split('/')[-1], d['value'], 'tok/s rows/step %.1f' % (s['decode_rows'] / s['decode_steps']))"
  done
done
unset RT_SKINNY_TN
timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 16 > $D/mb_b16.log 2>&1 && grep "^| skinny" $D/mb_b16.log
timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 3 > $D/mb_b3.log 2>&1 && grep "^| skinny" $D/mb_b3.log
