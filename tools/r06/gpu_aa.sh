#!/bin/bash
# round-6 GPU pass AA: B = 1 (sequential rounds) decode attention — the separate combine launch vs
# the in-launch combine by the last-arriving split (RT_ATTN_EXT_SPLITS=0), at 16 / 32 splits;
# then the sequential driver bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06aa
mkdir -p $D
export PYTHONUNBUFFERED=1
for ext in 2 0; do
  for sp in 32 16; do
    RT_ATTN_EXT_SPLITS=$ext timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 1 --splits $sp \
      --shared 25000:0,10000:0,40000:0 > $D/b1_ext${ext}_s$sp.log 2>&1 || { tail -20 $D/b1_ext${ext}_s$sp.log; exit 1; }
    echo "ext=$ext splits=$sp"; grep -h "^| decode attn grouped" $D/b1_ext${ext}_s$sp.log
  done
done
for ext in 2 0; do
  RT_ATTN_EXT_SPLITS=$ext timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --round-mode sequential \
    > $D/seq_ext$ext.json 2> $D/seq_ext$ext.err || { tail -20 $D/seq_ext$ext.err; exit 1; }
  echo "seq ext=$ext: $(python -c "import json;d=json.load(open('$D/seq_ext$ext.json'));print(d['value'], d['ms_per_step'])")"
done
