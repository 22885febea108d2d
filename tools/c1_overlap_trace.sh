#!/bin/bash
# 2-rank STRIPED rehearsal on one GPU (gloo world, knights of a table on different ranks), each
# rank under its own rocprofv3 kernel trace; then tools/c1_overlap.py correlates the C1 exchange
# windows with the kernels that ran inside them. Usage: tools/c1_overlap_trace.sh <out.md>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ROUNDTABLE_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 MASTER_PORT=29547 WORLD_SIZE=2 \
       OMP_NUM_THREADS=2 HSA_ENABLE_IPC_MODE_LEGACY=0 ROUNDTABLE_TRACE=1
rm -rf /tmp/c1tr && mkdir -p /tmp/c1tr gpurun_out
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv \
      -d /tmp/c1tr/r$r -o tr -- python3 bench.py --gpus 2 --scaling weak --placement striped \
      --model llama3-8b --layers 8 --new-tokens 128 --steps 4 --warmup 1 --kv-fraction 0.1 \
      --max-kv-tokens 131072 --c1-events /tmp/c1tr/ev > gpurun_out/c1tr_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
[ "$rc" -eq 0 ] || { echo "rank failed rc=$rc"; tail -20 gpurun_out/c1tr_r0.log gpurun_out/c1tr_r1.log; exit "$rc"; }
python3 tools/c1_overlap.py /tmp/c1tr/ev /tmp/c1tr/r0 /tmp/c1tr/r1 > "$1"
find /tmp/c1tr -name "*marker*" | head -3
for f in $(find /tmp/c1tr -name "*marker_api_trace.csv" | head -1); do head -5 "$f"; grep -c "speculative" "$f"; done
cat "$1"
