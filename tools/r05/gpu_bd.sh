#!/bin/bash
# round-5 GPU pass BD: serve load test with the K read order, old order (RT_ATTN_KPERM=0) as A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05bd
mkdir -p $D
export PYTHONUNBUFFERED=1
for kp in 0 1; do
  RT_ATTN_KPERM=$kp timeout -k 10 300 python -u tools/serve_bench.py --clients 32 --requests 96 --prompt-words 100 --max-tokens 256 \
    > $D/s32_kp$kp.log 2>&1 || { tail -20 $D/s32_kp$kp.log; exit 1; }
  python -c "
import json; d = json.loads(open('$D/s32_kp$kp.log').read().strip().splitlines()[-1]); s = d['scheduler']
print('KPERM=$kp', d['value'], 'tok/s p50', d['latency_s_p50'], 'p99', d['latency_s_p99'], 'rows/step %.1f' % (s['decode_rows'] / s['decode_steps']))"
done
