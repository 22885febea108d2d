#!/bin/bash
# round-5 GPU pass AZ: new K read order as the default — full GPU suite + smoke, then driver-config
# bench A/B/A/B (RT_ATTN_KPERM=0 = old order) and a sequential-rounds A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05az
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1 || { tail -30 $D/gpu_tests_full.log; exit 1; }
tail -1 $D/gpu_tests_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
for pass in 1 2; do
  for kp in 0 1; do
    RT_ATTN_KPERM=$kp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench_kp${kp}_$pass.json 2> $D/bench_kp${kp}_$pass.err \
      || { tail -20 $D/bench_kp${kp}_$pass.err; exit 1; }
    python -c "import json; d = json.loads(open('$D/bench_kp${kp}_$pass.json').read().strip().splitlines()[-1]); print('KPERM=$kp pass $pass', d['value'], d['ms_per_step'])"
  done
done
for kp in 0 1; do
  RT_ATTN_KPERM=$kp timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --round-mode sequential > $D/seq_kp$kp.json 2> $D/seq_kp$kp.err \
    || { tail -20 $D/seq_kp$kp.err; exit 1; }
  python -c "import json; d = json.loads(open('$D/seq_kp$kp.json').read().strip().splitlines()[-1]); print('sequential KPERM=$kp', d['value'], d['ms_per_step'])"
done
