#!/bin/bash
# round-5 GPU pass AY: decode attention K-row read order (RT_ATTN_KPERM) — tests, then A/B/A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05ay
mkdir -p $D
export PYTHONUNBUFFERED=1
RT_ATTN_KPERM=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "decode or attention" > $D/tests_kperm1.log 2>&1 || { tail -30 $D/tests_kperm1.log; exit 1; }
tail -1 $D/tests_kperm1.log
for pass in 1 2; do
  for kp in 0 1; do
    RT_ATTN_KPERM=$kp timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10 \
      --shared 22000:1500,40000:1500,6000:800 > $D/tp1_kp${kp}_$pass.log 2>&1 || exit 1
    RT_ATTN_KPERM=$kp timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 8 --batch 3 --splits 64 \
      --shared 22000:1500 > $D/tp8_kp${kp}_$pass.log 2>&1 || exit 1
    RT_ATTN_KPERM=$kp timeout -k 10 300 python -u tools/microbench.py --only attn --batch 1 --ctx 25000 --splits 32 \
      > $D/b1_kp${kp}_$pass.log 2>&1 || exit 1
    echo "KPERM=$kp pass $pass"; grep -h "^| decode attn" $D/tp1_kp${kp}_$pass.log $D/tp8_kp${kp}_$pass.log $D/b1_kp${kp}_$pass.log | grep -v "ctx=1500"
  done
done
