#!/bin/bash
# A/B timing of libnavenv builds on one GPU box: bench.py (timed region, no events) with each
# NAV_LIB in turn, interleaved, `rounds` times. usage: tools/ab.sh rounds lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq "$rounds"); do
  for l in "$@"; do
    out=$(NAV_LIB=$l timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-timed-events 2>/dev/null | tail -1)
    rc=$?
    echo "$(basename "$l") $out" | tee -a gpurun_out/ab.log
    if [ "$rc" -ne 0 ]; then exit "$rc"; fi
  done
done
