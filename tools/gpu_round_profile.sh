# One GPU call (run through gpurun from the repo root): rebuild libnavenv + the oracle from source
# on the box, the GPU test suite, smoke(), the default bench line, then the rocprofv3 evidence for it:
# kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes (separate, TCC slots), the SQ pass
# (MFMA busy), and a kernel trace of the 65 536-env step-kernel sweep.
# usage: bash tools/gpu_round_profile.sh TAG
set -e -o pipefail
TAG=${1:-r02x}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
BENCH_SHORT="--steps 20 --warmup 3 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0"
timeout -k 10 600 make -B -j16 -C residual-td3-robot-navigation_amd > "$O/box_build.log" 2>&1
timeout -k 10 120 make -B -C oracle >> "$O/box_build.log" 2>&1
echo "rebuilt from source on $(hostname) $(date -u)" >> "$O/box_build.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gputest.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python bench.py $BENCH_SHORT > "$O/trace.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > "$O/fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > "$O/write.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/sq" -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > "$O/sq.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/sweep_trace" -o run -- python bench.py --sweep-only 65536 > "$O/sweep_trace.log" 2>&1
echo done > "$O/DONE"
