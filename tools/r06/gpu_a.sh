#!/bin/bash
# round-6 GPU pass A: (1) the fused-MLP phase-1 anomaly apart (sync forms), (2) decode attention
# K/V load modes (RT_ATTN_LM: 1 = nt loads, 2 = chunk-major K addressing probe, 3 = both)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06a
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/probes/fused_mlp_tp.py --tp 8,4 > $D/fused_mlp.log 2>&1 || { tail -20 $D/fused_mlp.log; exit 1; }
grep '^{"tp"' $D/fused_mlp.log
RT_ATTN_LM=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "decode" > $D/tests_lm1.log 2>&1 || { tail -30 $D/tests_lm1.log; exit 1; }
tail -1 $D/tests_lm1.log
for pass in 1 2; do
  for lm in 0 1 2 3; do
    RT_ATTN_LM=$lm timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 \
      --shared 22000:1500,40000:1500,6000:800 > $D/tp1_lm${lm}_$pass.log 2>&1 || exit 1
    RT_ATTN_LM=$lm timeout -k 10 300 python -u tools/microbench.py --only attn --batch 1 --ctx 25000 --splits 32 \
      > $D/b1_lm${lm}_$pass.log 2>&1 || exit 1
    echo "LM=$lm pass $pass"; grep -h "^| decode attn" $D/tp1_lm${lm}_$pass.log $D/b1_lm${lm}_$pass.log | grep -v "ctx=1500"
  done
done
