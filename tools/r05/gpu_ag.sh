#!/bin/bash
# round-5 GPU pass AG: full GPU suite + smoke + driver-config bench (N = 1) on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ag
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1; rc=$?
tail -3 $D/gpu_tests_full.log
grep -E "FAILED|ERROR" $D/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --out $D/bench1.json > $D/bench1.log 2>&1 || { tail -20 $D/bench1.log; exit 1; }
python -c "import json; d=json.load(open('$D/bench1.json')); print(d['value'], d['ms_per_round'], d['detail']['failed_turns'])"
