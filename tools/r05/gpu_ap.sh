#!/bin/bash
# round-5 GPU pass AP: sequential (reference-semantics) rounds on the final tree, kernel table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05ap
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/seq -o p -- \
  python3 bench.py --round-mode sequential --steps 20 --warmup 5 --out $D/seq_bench.json > $D/seq.log 2>&1 || { tail -20 $D/seq.log; exit 1; }
python3 tools/prof_summary.py $D/seq $D/seq_kernels.md --drop-trace
head -12 $D/seq_kernels.md
python3 -c "import json; d=json.load(open('$D/seq_bench.json')); print('sequential under profiler', d['value'], d['ms_per_round'], d['detail']['engine_decode_ms_per_round'])"
