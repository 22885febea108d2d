#!/bin/bash
# round-6 GPU pass AH: the driver-config bench, three passes on one more box (the spread record)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06ah
mkdir -p $D
export PYTHONUNBUFFERED=1
for pass in 1 2 3; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench_$pass.json 2> $D/bench_$pass.err || { tail -20 $D/bench_$pass.err; exit 1; }
  echo "bench $pass: $(python -c "import json;d=json.load(open('$D/bench_$pass.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'])")"
done
