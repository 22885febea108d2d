#!/bin/bash
# round-5 GPU pass BC: kernel table of the driver-config bench on the final tree (K read order on)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r05bc
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof1 -o p -- \
  python3 bench.py --steps 20 --warmup 5 --out $D/bench.json > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
python3 tools/prof_summary.py $D/prof1 $D/prof1_kernels.md --drop-trace
head -12 $D/prof1_kernels.md
python3 -c "import json; d=json.load(open('$D/bench.json')); print('driver config under profiler', d['value'], d['ms_per_round'], d['detail']['engine_decode_ms_per_round'])"
