#!/bin/bash
# round-6 GPU pass C: decode attention knobs on the chunk-major K layout (nt per operand, splits,
# XCD order + plain partials, in-launch combine, latency probes, tp 8 shard, ungrouped rows), then
# sequential rounds (B = 1) base vs new
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06c
mkdir -p $D
export PYTHONUNBUFFERED=1
mb() {  # name, env..., -- microbench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 300 python -u tools/microbench.py "$@" > $D/$name.log 2>&1 || { tail -5 $D/$name.log; return 1; }
  echo "== $name"; grep -h "^| decode attn" $D/$name.log | grep -v "ctx=1500"
}
G="--only gattn --tp 1 --batch 3 --shared 22000:1500,40000:1500"
for lm in 0 1 2 3; do mb g_lm$lm RT_ATTN_LM=$lm -- $G --splits 10 || exit 1; done
mb g_splits RT_X=0 -- $G --splits 8,12 || exit 1
mb g_xcd RT_ATTN_XCD=1 RT_ATTN_PLAIN_PARTIALS=1 -- $G --splits 8 || exit 1
mb g_xcd10 RT_ATTN_XCD=1 -- $G --splits 10 || exit 1
mb g_inlaunch RT_ATTN_EXT_SPLITS=0 -- $G --splits 10 || exit 1
mb g_probe1 RT_ATTN_PROBE=1 -- $G --splits 10 || exit 1
mb g_probe2 RT_ATTN_PROBE=2 -- $G --splits 10 || exit 1
mb g_nocomb RT_ATTN_SKIP_COMBINE=1 -- $G --splits 10 || exit 1
for lm in 0 3; do
  mb tp8_lm$lm RT_ATTN_LM=$lm -- --only gattn --tp 8 --batch 3 --splits 64 --shared 22000:1500 || exit 1
  mb priv3_lm$lm RT_ATTN_LM=$lm -- --only attn --batch 3 --ctx 25000 --splits 10 || exit 1
  mb priv16_lm$lm RT_ATTN_LM=$lm -- --only attn --batch 16 --ctx 2000 --splits 2 || exit 1
done
timeout -k 10 600 python -u ab_base/bench.py --steps 20 --warmup 5 --round-mode sequential > $D/seq_base.json 2> $D/seq_base.err || { tail -20 $D/seq_base.err; exit 1; }
echo "seq base: $(python -c "import json;d=json.load(open('$D/seq_base.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --round-mode sequential > $D/seq_new.json 2> $D/seq_new.err || { tail -20 $D/seq_new.err; exit 1; }
echo "seq new: $(python -c "import json;d=json.load(open('$D/seq_new.json'));print(d['value'], d['ms_per_step'])")"
