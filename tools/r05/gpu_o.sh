#!/bin/bash
# round-5 GPU pass O: which sampler branch decides each row on real decode logits, and its cost
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r05o
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/probes/sampler_paths.py --mode gen --logits $D/logits.pt && \
RT_SMP_PROBE=5 timeout -k 10 200 python -u tools/probes/sampler_paths.py --mode paths --logits $D/logits.pt --out $D/paths.json && \
timeout -k 10 300 python -u tools/probes/sampler_paths.py --mode times --logits $D/logits.pt --paths $D/paths.json --out $D/times.json
