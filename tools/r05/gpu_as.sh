#!/bin/bash
# round-5 GPU pass AS: serve with the new default batch (32) — GPU serve tests + load test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05as
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_serve.py tests/test_serve_tp.py tests/test_cli_gpu.py -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -m gpu > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for mb in 16 32; do
  timeout -k 10 300 python -u tools/serve_bench.py --clients 32 --requests 96 --prompt-words 100 --max-tokens 256 --max-batch $mb \
    > $D/s32_mb$mb.log 2>&1 || { tail -20 $D/s32_mb$mb.log; exit 1; }
  python -c "
import json; d = json.loads(open('$D/s32_mb$mb.log').read().strip().splitlines()[-1]); s = d['scheduler']
print('max_batch $mb', d['value'], 'tok/s p50', d['latency_s_p50'], 'p99', d['latency_s_p99'], 'rows/step %.1f' % (s['decode_rows'] / s['decode_steps']))"
done
