#!/bin/bash
# round-6 GPU pass Y: the final tree (LDS-DMA attention knob, Qwen2 family, context guard) —
# full GPU suite, smoke, serve 64 clients, driver-config bench x2, sequential rounds, kernel table under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06y
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > $D/gpu_tests_full.log 2>&1; rc=$?
tail -1 $D/gpu_tests_full.log
grep -E "FAILED|ERROR" $D/gpu_tests_full.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python -u tools/serve_bench.py --clients 64 --requests 192 --prompt-words 100 --max-tokens 256 \
  --max-batch 64 > $D/serve_c64.log 2>&1 || { tail -20 $D/serve_c64.log; exit 1; }
echo "serve 64: $(grep '^{' $D/serve_c64.log | cut -c1-300)"
for pass in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_$pass.json 2> $D/bench_$pass.err || { tail -20 $D/bench_$pass.err; exit 1; }
  echo "bench $pass: $(python -c "import json;d=json.load(open('$D/bench_$pass.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --round-mode sequential > $D/seq.json 2> $D/seq.err || { tail -20 $D/seq.err; exit 1; }
echo "seq: $(python -c "import json;d=json.load(open('$D/seq.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof1 -o p -- \
  python3 bench.py --steps 20 --warmup 5 --out $D/prof1_bench.json > $D/prof1.log 2>&1 || { tail -20 $D/prof1.log; exit 1; }
python3 tools/prof_summary.py $D/prof1 $D/prof1_kernels.md --drop-trace
head -9 $D/prof1_kernels.md
