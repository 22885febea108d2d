#!/bin/bash
# round-6 GPU pass X: Qwen2.5-7B / 0.5B at the driver's table shape (3 knights, shared layout,
# parallel rounds), 10 timed + 3 warm-up rounds: contexts stay inside Qwen2.5's 32768 positions
# (pass W's 25-round run crossed them and read past the RoPE table; the engine now fails such a
# turn on the host, tests/test_engine_cpu.py::test_context_past_max_positions_fails_the_turn_on_the_host)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/r06x
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --model qwen2.5-7b --steps 10 --warmup 3 > $D/bench_qwen7b.json \
  2> $D/bench_qwen7b.err || { tail -20 $D/bench_qwen7b.err; exit 1; }
echo "qwen2.5-7b: $(python -c "import json;d=json.load(open('$D/bench_qwen7b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'], d['config']['seq_len'])")"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $D/bench_llama8b.json \
  2> $D/bench_llama8b.err || { tail -20 $D/bench_llama8b.err; exit 1; }
echo "llama3-8b (same rounds): $(python -c "import json;d=json.load(open('$D/bench_llama8b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'], d['config']['seq_len'])")"
timeout -k 10 400 python -u bench.py --model qwen2.5-0.5b --steps 10 --warmup 3 > $D/bench_qwen05b.json \
  2> $D/bench_qwen05b.err || { tail -20 $D/bench_qwen05b.err; exit 1; }
echo "qwen2.5-0.5b: $(python -c "import json;d=json.load(open('$D/bench_qwen05b.json'));print(d['value'], d['ms_per_step'], d['detail']['failed_turns'], d['config']['seq_len'])")"
