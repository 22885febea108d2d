#!/bin/bash
# round-5 GPU pass W: serving throughput (roundtable serve under concurrent clients) on the round-5 tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05w
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/serve_bench.py --clients 16 --requests 32 --prompt-words 400 --max-tokens 256 --max-batch 16 > $D/s16_256.log 2>&1 || { tail -20 $D/s16_256.log; exit 1; }
tail -1 $D/s16_256.log
timeout -k 10 400 python -u tools/serve_bench.py --clients 16 --requests 16 --prompt-words 100 --max-tokens 512 --max-batch 16 > $D/s16_512.log 2>&1 || { tail -20 $D/s16_512.log; exit 1; }
tail -1 $D/s16_512.log
timeout -k 10 400 python -u tools/serve_bench.py --clients 32 --requests 64 --prompt-words 100 --max-tokens 256 --max-batch 32 > $D/s32_256.log 2>&1 || { tail -20 $D/s32_256.log; exit 1; }
tail -1 $D/s32_256.log
timeout -k 10 300 python -u tools/microbench.py --only gemm --batch 16 > $D/mb_gemm16.log 2>&1 || { tail -20 $D/mb_gemm16.log; exit 1; }
grep "^|" $D/mb_gemm16.log | head -20
