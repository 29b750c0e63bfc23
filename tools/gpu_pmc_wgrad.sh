set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/r02i_pmc -o run -- python tools/wgrad_bench.py --reps 5 > gpurun_out/r02i_pmc.log 2>&1
