#!/bin/bash
# round-6 GPU pass N: round-end rehearsal of the driver's checks on the final tree — GPU suite,
# smoke, serve load (zero-loss, 64-row default), bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06n
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1; rc=$?
tail -1 $D/gpu_tests_full.log
grep -E "FAILED|ERROR" $D/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python -u tools/serve_bench.py --clients 64 --requests 192 --prompt-words 100 --max-tokens 256 \
  --max-batch 64 > $D/serve_c64.log 2>&1; rc=$?
echo "serve 64 rc=$rc: $(grep '^{' $D/serve_c64.log | cut -c1-400)"
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
echo "bench (defaults): $(cat $D/bench_default.json)"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
echo "bench: $(python -c "import json;d=json.load(open('$D/bench.json'));print(d['value'], d['ms_per_step'])")"
