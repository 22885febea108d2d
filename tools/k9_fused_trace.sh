#!/bin/bash
# 2-rank tensor-parallel rehearsal on ONE GPU (gloo world, strong-scaling bench, Llama-3-8B shapes,
# 8 layers) with the fused row-parallel GEMM + one-shot all-reduce FORCED (ROUNDTABLE_FUSED_AR=1)
# and each rank under its own rocprofv3 kernel trace: shows which K9 kernels the decode graph runs
# (skinny_gemm_ar_kernel for o / down, oneshot_ag_kernel for the logits) and their per-call times.
# Timing caveat: two processes share the GPU, so the fused grids co-schedule badly (see
# profiles/r03/k9_fused_gather_shared_gpu.md). Usage: tools/k9_fused_trace.sh <out_prefix>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ROUNDTABLE_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 MASTER_PORT=29557 WORLD_SIZE=2 \
       OMP_NUM_THREADS=2 HSA_ENABLE_IPC_MODE_LEGACY=0 ROUNDTABLE_FUSED_AR="${ROUNDTABLE_FUSED_AR:-1}"
rm -rf /tmp/k9tr && mkdir -p /tmp/k9tr gpurun_out
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d /tmp/k9tr/r$r -o tr -- python3 bench.py --gpus 2 --model llama3-8b --layers 8 --new-tokens 64 \
      --steps 2 --warmup 1 --kv-fraction 0.1 --max-kv-tokens 65536 > gpurun_out/k9tr_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
[ "$rc" -eq 0 ] || { echo "rank failed rc=$rc"; tail -20 gpurun_out/k9tr_r0.log gpurun_out/k9tr_r1.log; exit "$rc"; }
for r in 0 1; do python3 tools/prof_summary.py /tmp/k9tr/r$r "$1_r$r.md" --drop-trace; done
grep -h '"metric"' gpurun_out/k9tr_r0.log | head -1 > "$1_bench.json"
head -12 "$1_r0.md"
