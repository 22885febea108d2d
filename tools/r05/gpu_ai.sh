#!/bin/bash
# round-5 GPU pass AI: kernel profile of config 3 (8 Mistral-7B knights batched on one GPU) and of a
# 16-row fixed batch (serving-batch GEMMs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05ai
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/cfg3 -o p -- \
  python3 bench.py --model mistral-7b --knights-per-table 8 --knights-per-gpu 8 --steps 4 --warmup 1 --out $D/cfg3.json > $D/cfg3.log 2>&1 \
  || { echo "cfg3 prof failed"; tail -20 $D/cfg3.log; exit 1; }
python3 tools/prof_summary.py $D/cfg3 $D/cfg3_kernels.md --drop-trace
head -12 $D/cfg3_kernels.md
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/b16 -o p -- \
  python3 bench.py --knights-per-table 16 --steps 3 --warmup 1 --new-tokens 256 --out $D/b16.json > $D/b16.log 2>&1 \
  || { echo "b16 prof failed"; tail -20 $D/b16.log; exit 1; }
python3 tools/prof_summary.py $D/b16 $D/b16_kernels.md --drop-trace
head -12 $D/b16_kernels.md
