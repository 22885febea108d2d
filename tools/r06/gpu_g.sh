#!/bin/bash
# round-6 GPU pass G: final tree — full GPU suite, smoke, driver-config bench A/B/A/B against the
# round-5 tree, sequential rounds, BASELINE configs 3 / 4 / 16 knights, the bench under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06g
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1; rc=$?
tail -3 $D/gpu_tests_full.log
grep -E "FAILED|ERROR" $D/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
for pass in 1 2; do
  timeout -k 10 400 python -u ab_base/bench.py --steps 20 --warmup 5 > $D/bench_base_$pass.json 2> $D/bench_base_$pass.err || { tail -20 $D/bench_base_$pass.err; exit 1; }
  echo "base $pass: $(python -c "import json;d=json.load(open('$D/bench_base_$pass.json'));print(d['value'], d['ms_per_step'])")"
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_new_$pass.json 2> $D/bench_new_$pass.err || { tail -20 $D/bench_new_$pass.err; exit 1; }
  echo "new  $pass: $(python -c "import json;d=json.load(open('$D/bench_new_$pass.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --round-mode sequential > $D/seq_new.json 2> $D/seq_new.err || { tail -20 $D/seq_new.err; exit 1; }
echo "seq new: $(python -c "import json;d=json.load(open('$D/seq_new.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 500 python -u tools/run_configs.py --config 3 > $D/cfg3.log 2>&1 || { tail -20 $D/cfg3.log; exit 1; }
echo "cfg3: $(grep '^{' $D/cfg3.log | tail -1 | cut -c1-200)"
timeout -k 10 500 python -u tools/run_configs.py --config 4 > $D/cfg4.log 2>&1 || { tail -20 $D/cfg4.log; exit 1; }
echo "cfg4: $(grep '^{' $D/cfg4.log | tail -1 | cut -c1-300)"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --knights-per-table 16 --new-tokens 256 > $D/b16.json 2> $D/b16.err || { tail -20 $D/b16.err; exit 1; }
echo "16 knights: $(python -c "import json;d=json.load(open('$D/b16.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof1 -o p -- \
  python3 bench.py --steps 20 --warmup 5 --out $D/prof1_bench.json > $D/prof1.log 2>&1 || { tail -20 $D/prof1.log; exit 1; }
python3 tools/prof_summary.py $D/prof1 $D/prof1_kernels.md --drop-trace
head -9 $D/prof1_kernels.md
python3 -c "import json; d=json.load(open('$D/prof1_bench.json')); print('bench under profiler', d['value'], d['ms_per_round'])"
