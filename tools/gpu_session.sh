#!/bin/bash
# One gpurun session: each GPU step under its own time limit; stop at the first crash/timeout.
# Usage: tools/gpu_session.sh "<name>:<timeout_s>:<command>" ...
# A step's exit code 0/1 (pass / test failures) continues; anything else (abort 134, segv 139,
# timeout 124/137, ...) ends the session so nothing more touches a possibly-faulted GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${tmo}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "=== stopping session after [$name] rc=$rc" | tee -a gpurun_out/session.log
    exit "$rc"
  fi
done
exit 0
