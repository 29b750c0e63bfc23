#!/bin/bash
# A/B timing on one GPU box: bench.py (timed region, no events) under each environment setting
# in turn (e.g. NAV_LIB=path/to/lib.so or NAV_CRITIC_ROW_BWD=0), interleaved, `rounds` times.
# usage: tools/ab.sh rounds "VAR=value ..." "VAR=value ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq "$rounds"); do
  for v in "$@"; do
    out=$(env $v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-timed-events 2>/dev/null | tail -1)
    rc=$?
    echo "[$v] $out" | tee -a gpurun_out/ab.log
    if [ "$rc" -ne 0 ]; then exit "$rc"; fi
  done
done
