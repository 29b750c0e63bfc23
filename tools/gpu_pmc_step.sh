set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r02q_pmc -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sweep --no-utd-sweep --long-steps 0 > gpurun_out/r02q_pmc.log 2>&1
