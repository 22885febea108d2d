#!/bin/bash
# round-6 GPU pass D: tree with nt on every attention launch — full GPU suite, smoke, the
# driver-config bench under rocprofv3, then the serve load tests (zero-loss check, streaming TTFC)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06d
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1; rc=$?
tail -3 $D/gpu_tests_full.log
grep -E "FAILED|ERROR" $D/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof1 -o p -- \
  python3 bench.py --steps 20 --warmup 5 --out $D/prof1_bench.json > $D/prof1.log 2>&1 || { tail -20 $D/prof1.log; exit 1; }
python3 tools/prof_summary.py $D/prof1 $D/prof1_kernels.md --drop-trace
head -8 $D/prof1_kernels.md
python3 -c "import json; d=json.load(open('$D/prof1_bench.json')); print('bench under profiler', d['value'], d['ms_per_round'])"
for c in "32 96" "64 192"; do
  set -- $c
  timeout -k 10 400 python -u tools/serve_bench.py --clients $1 --requests $2 --prompt-words 100 --max-tokens 256 \
    --max-batch 32 > $D/serve_c$1.log 2>&1; rc=$?
  echo "serve clients $1 rc=$rc: $(grep '^{' $D/serve_c$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'tok/s', d['completed_requests'], 'done', d['failed_requests'], 'failed', d['latency_s_p50'], d['latency_s_p99'])")"
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 400 python -u tools/serve_bench.py --clients 16 --requests 48 --prompt-words 100 --max-tokens 256 \
  --max-batch 32 --stream > $D/serve_stream.log 2>&1; rc=$?
echo "serve stream rc=$rc: $(grep '^{' $D/serve_stream.log)"
