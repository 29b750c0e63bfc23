#!/bin/bash
# One gpurun call: GPU parity tests, smoke, a short bench. Every GPU step has its own time limit;
# a fault / abort / timeout (exit status other than 0 or 1) ends the call there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/status.txt
run() {
  local name=$1 t=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/status.txt
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    tests) run gpu_tests 1200 python -m pytest tests -q -m gpu -x -p no:cacheprovider ;;
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run bench 600 python bench.py --steps 10 --warmup 3 --cpu-budget 8 ;;
    micro) run micro 600 python tools/microbench.py ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sweep ;;
    pmc) run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -T -f csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sweep &&
         run pmc_write 900 rocprofv3 --pmc WRITE_SIZE -T -f csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sweep &&
         run pmc_step_fetch 600 rocprofv3 --pmc FETCH_SIZE -T -f csv -d gpurun_out/pmc_step_fetch -o run -- python bench.py --sweep-only 16777216 &&
         run pmc_step_write 600 rocprofv3 --pmc WRITE_SIZE -T -f csv -d gpurun_out/pmc_step_write -o run -- python bench.py --sweep-only 16777216 ;;
    pmcmicro) run pmc_micro_a 900 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -T -f csv -d gpurun_out/pmc_micro_a -o run -- python tools/microbench.py --quick ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
