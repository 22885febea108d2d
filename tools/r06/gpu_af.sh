#!/bin/bash
# round-6 GPU pass AF: the final commit again (after the padded-slot prefill) — full GPU suite,
# smoke, driver-config bench x2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06af
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1; rc=$?
tail -1 $D/gpu_tests_full.log
grep -E "FAILED|ERROR" $D/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
for pass in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_$pass.json 2> $D/bench_$pass.err || { tail -20 $D/bench_$pass.err; exit 1; }
  echo "bench $pass: $(python -c "import json;d=json.load(open('$D/bench_$pass.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
done
