#!/bin/bash
# round-6 GPU pass M: 16-wave grouped attention workgroups (RT_ATTN_W16) vs the 8-wave default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06m
mkdir -p $D
export PYTHONUNBUFFERED=1
G="--only gattn --tp 1 --batch 3 --shared 22000:1500,40000:1500,6000:800"
for pass in 1 2; do
  timeout -k 10 300 python -u tools/microbench.py $G --splits 10 > $D/w8_$pass.log 2>&1 || exit 1
  RT_ATTN_W16=1 timeout -k 10 300 python -u tools/microbench.py $G --splits 4,5,6 > $D/w16_$pass.log 2>&1 || exit 1
  echo "pass $pass"; grep -h "^| decode attn grouped" $D/w8_$pass.log $D/w16_$pass.log
done
RT_ATTN_W16=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "shared_prefix" > $D/tests_w16.log 2>&1; tail -1 $D/tests_w16.log
