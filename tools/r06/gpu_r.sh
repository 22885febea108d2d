#!/bin/bash
# round-6 GPU pass R: kernel tables of the final tree for sequential rounds (B = 1) and the
# simulated tp 8 shard with 5-us device-simulated collectives
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r06r
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/seq -o p -- \
  python3 bench.py --steps 5 --warmup 2 --round-mode sequential --out $D/seq_bench.json > $D/seq.log 2>&1 || { tail -20 $D/seq.log; exit 1; }
python3 tools/prof_summary.py $D/seq $D/prof_sequential_kernels.md --drop-trace
head -9 $D/prof_sequential_kernels.md | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/tp8 -o p -- \
  python3 bench.py --simulate-tp 8 --sim-k9-us 5 --steps 5 --warmup 2 --out $D/prof8_bench.json > $D/tp8.log 2>&1 || { tail -20 $D/tp8.log; exit 1; }
python3 tools/prof_summary.py $D/tp8 $D/prof8_sim_comm5_kernels.md --drop-trace
head -10 $D/prof8_sim_comm5_kernels.md | cut -c1-200
