#!/bin/bash
# round-5 GPU pass Q: XCD-aware attention / combine item order + plain (L2-resident) partials:
# numerics first (decode attention GPU tests with both knobs on), then an A/B/A/B microbench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05q
mkdir -p $D
export PYTHONUNBUFFERED=1
RT_ATTN_XCD=1 RT_ATTN_PLAIN_PARTIALS=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "decode or paged or group" > $D/tests_xcd_plain.log 2>&1 \
  || { echo "tests failed"; tail -30 $D/tests_xcd_plain.log; exit 1; }
tail -1 $D/tests_xcd_plain.log
for pass in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    RT_ATTN_XCD=$1 RT_ATTN_PLAIN_PARTIALS=$2 timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1,2 \
      --shared 22000:1500,40000:1500,6000:800 --splits 8,16 > $D/mb_x$1_p$2_pass$pass.log 2>&1 \
      || { echo "microbench failed"; tail -20 $D/mb_x$1_p$2_pass$pass.log; exit 1; }
    echo "xcd=$1 plain=$2 pass $pass"; grep "^| decode attn grouped" $D/mb_x$1_p$2_pass$pass.log
  done
done
