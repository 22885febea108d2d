#!/bin/bash
# round-5 GPU pass AW: final-tree driver-config bench (two passes) and sequential rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05aw
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench_$pass.json 2> $D/bench_$pass.err || { tail -20 $D/bench_$pass.err; exit 1; }
  python -c "import json; d = json.loads(open('$D/bench_$pass.json').read().strip().splitlines()[-1]); print('pass $pass', d['value'], d['ms_per_step'])"
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --round-mode sequential > $D/bench_seq.json 2> $D/bench_seq.err || { tail -20 $D/bench_seq.err; exit 1; }
python -c "import json; d = json.loads(open('$D/bench_seq.json').read().strip().splitlines()[-1]); print('sequential', d['value'], d['ms_per_step'])"
