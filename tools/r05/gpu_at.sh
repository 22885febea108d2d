#!/bin/bash
# Grouped decode attention at tp 1, B = 3: one workgroup per CU (10 splits) vs two (16-21 splits)
set -o pipefail
mkdir -p gpurun_out/r05at
timeout -k 10 300 python -u tools/microbench.py --only gattn --tp 1 --batch 3 --splits 10,16,20,21 \
  --shared 22000:1500,40000:1500,6000:800 > gpurun_out/r05at/gattn_tp1_occ.log 2>&1
