#!/bin/bash
# round-5 GPU pass H: kernel profiles — tp1 at the driver config, simulated tp8 with device-simulated comm
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05h
export PYTHONUNBUFFERED=1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05h/prof1 -o p -- \
  python3 bench.py --steps 20 --warmup 5 --out gpurun_out/r05h/prof1_bench.json > gpurun_out/r05h/prof1.log 2>&1 \
  || { echo "prof1 failed"; tail -20 gpurun_out/r05h/prof1.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/r05h/prof1 gpurun_out/r05h/prof1_kernels.md --drop-trace
head -14 gpurun_out/r05h/prof1_kernels.md
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05h/prof8 -o p -- \
  python3 bench.py --simulate-tp 8 --sim-k9-us 5 --steps 5 --warmup 2 --out gpurun_out/r05h/prof8_bench.json > gpurun_out/r05h/prof8.log 2>&1 \
  || { echo "prof8 failed"; tail -20 gpurun_out/r05h/prof8.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/r05h/prof8 gpurun_out/r05h/prof8_kernels.md --drop-trace
head -14 gpurun_out/r05h/prof8_kernels.md
