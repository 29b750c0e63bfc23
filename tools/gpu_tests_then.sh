#!/bin/bash
# One gpurun call: the named GPU test files first (fast feedback), then the whole GPU suite and
# the requested gpu_check.sh steps. Each step has its own time limit; a fault ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FIRST=${FIRST:-}
if [ -n "$FIRST" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/first.log 2>&1
  rc=$?; echo "first rc=$rc" | tee -a gpurun_out/status.txt
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
fi
exec_steps="$*"
if [ -n "$exec_steps" ]; then bash tools/gpu_check.sh $exec_steps; fi
