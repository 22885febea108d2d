#!/bin/bash
# round-6 GPU pass Z: pass Y without the suite (305 of 306 passed there): the one failed rehearsal test
# full GPU suite, smoke, serve 64 clients, driver-config bench x2, sequential rounds, kernel table under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06z
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest "tests/test_distributed_gpu.py::test_fused_ar_correct_at_tp4_tp8_with_cu_split_on_shared_gpu" \
  tests/test_hf_parity.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gpu_tests_rerun.log 2>&1; rc=$?
tail -1 $D/gpu_tests_rerun.log
grep -E "FAILED|ERROR|expired" $D/gpu_tests_rerun.log | head -10
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
