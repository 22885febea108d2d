#!/bin/bash
# round-6 GPU pass O: long context — 45 rounds (contexts to ~75K tokens per knight), round-5 tree
# vs final tree on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06o
mkdir -p $D
export PYTHONUNBUFFERED=1
for t in new base; do
  dir=.; [ $t = base ] && dir=ab_base
  timeout -k 10 500 python -u $dir/bench.py --steps 40 --warmup 5 > $D/long45_$t.json 2> $D/long45_$t.err || { tail -20 $D/long45_$t.err; exit 1; }
  echo "$t: $(python -c "import json;d=json.load(open('$D/long45_$t.json'));print(d['value'], d['ms_per_round'], d['config'].get('seq_len'), d['detail']['failed_turns'])")"
done
