#!/bin/bash
# round-5 GPU pass AV: fused decode up to 64 rows (four 16-row blocks per weight fragment) —
# GEMM / RoPE / fused-decode tests at 33..64 rows, GEMM timings, fixed-batch decode A/B, serve
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05av
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "serving_batch or rope_epilogue or rope_serving or odd_tile" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for m in 64 48; do
  timeout -k 10 300 python -u tools/microbench.py --only gemm --batch $m > $D/mb_b$m.log 2>&1 || exit 1
done
RT_SKINNY_TNS=0 timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 64 > $D/mb_b64_tns0.log 2>&1 || exit 1
grep -h "^| " $D/mb_b*.log | grep -v "op |\|---" || true
for pass in 1 2; do
  for rows in 32 64; do
    ROUNDTABLE_FUSED_ROWS=$rows timeout -k 10 400 python -u bench.py --knights-per-table 64 --new-tokens 256 --steps 3 --warmup 1 \
      > $D/b64_fused${rows}_$pass.json 2> $D/b64_fused${rows}_$pass.err || { tail -20 $D/b64_fused${rows}_$pass.err; exit 1; }
    python -c "
import json; d = json.loads(open('$D/b64_fused${rows}_$pass.json').read().strip().splitlines()[-1])
print('64 knights, fused rows $rows, pass $pass:', d['value'], 'tok/s', d['detail'].get('engine_decode_ms_per_round'), 'ms decode/round')"
  done
done
for mb in 32 64; do
  timeout -k 10 400 python -u tools/serve_bench.py --clients 64 --requests 192 --prompt-words 100 --max-tokens 256 --max-batch $mb \
    > $D/s64_mb$mb.log 2>&1 || { tail -20 $D/s64_mb$mb.log; exit 1; }
  python -c "
import json; d = json.loads(open('$D/s64_mb$mb.log').read().strip().splitlines()[-1]); s = d['scheduler']
print('64 clients, max_batch $mb', d['value'], 'tok/s p50', d['latency_s_p50'], 'p99', d['latency_s_p99'], 'rows/step %.1f' % (s['decode_rows'] / s['decode_steps']))"
done
