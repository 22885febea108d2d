#!/bin/bash
# Round-4 measurement session on one MI355X (tools/gpu_session.sh semantics: each step under its
# own time limit, the session stops at the first crash / timeout). Usage:
#   tools/r04_measure.sh <step>...   steps: probes tests sims seq bench prof smp capture persist k9 host
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
steps=()
for s in "$@"; do
  case "$s" in
    probes) steps+=("overlap:60:build/probes/overlap_probe"
                    "mb_tp:200:python -u tools/microbench.py --only gemm_tp,gattn --tp 2,4,8 --splits 16,32,64") ;;
    tests) steps+=("gputests:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/") ;;
    sims) for n in 8 4 2; do
            steps+=("sim$n:150:python -u bench.py --simulate-tp $n --steps 20 --warmup 5 --out gpurun_out/r04/sim$n.json")
          done ;;
    seq) for n in 8 4 2; do
           steps+=("simseq$n:300:python -u bench.py --simulate-tp $n --round-mode sequential --steps 20 --warmup 5 --out gpurun_out/r04/sim${n}_seq.json")
         done
         steps+=("seq1:400:python -u bench.py --round-mode sequential --steps 20 --warmup 5 --out gpurun_out/r04/sim1_seq.json") ;;
    bench) steps+=("bench1:200:python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r04/sim1.json") ;;
    smp) steps+=("smp:120:python -u tools/sampler_probe.py") ;;
    persist) steps+=("pp8:300:python -u tools/probes/persistent_tp8.py --ctx 8192 --layers 8 --splits 16,32,64") ;;
    k9) steps+=("osb2:200:ROUNDTABLE_DIST_BACKEND=gloo ROUNDTABLE_FUSED_AR=probe python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 tools/oneshot_check.py --bench") ;;
    host) steps+=("ph:200:python -u tools/probes/prefill_host.py"
                  "hprof:300:python tools/probes/host_profile.py --out gpurun_out/r04/host_profile_sim8.txt -- --simulate-tp 8 --steps 3 --warmup 1") ;;
    capture) steps+=("capture:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_distributed_gpu.py -k 'captured or config5'") ;;
    prof) for n in 8 1; do
            if [ "$n" = 1 ]; then a=""; else a="--simulate-tp $n"; fi
            steps+=("prof$n:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/prof$n -o p -- python3 bench.py $a --steps 5 --warmup 2 && python3 tools/prof_summary.py gpurun_out/r04/prof$n gpurun_out/r04/prof${n}_kernels.md --drop-trace")
          done ;;
  esac
done
tools/gpu_session.sh "${steps[@]}"
