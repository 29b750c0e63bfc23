#!/bin/bash
# One gpurun call: rocprofv3 kernel trace + stats of a short bench, then one SQ counter pass
# (MFMA busy, instruction mix). usage: bash tools/gpu_prof_quick.sh TAG
set -e -o pipefail
TAG=${1:-r03x}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
SHORT="--steps 20 --warmup 3 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python bench.py $SHORT > "$O/trace.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/sq" -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > "$O/sq.log" 2>&1
echo done > "$O/DONE"
