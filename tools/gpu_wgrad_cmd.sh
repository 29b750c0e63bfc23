set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python tools/wgrad_bench.py > gpurun_out/r02c_wgrad.json
timeout -k 10 120 python tools/wgrad_bench.py --splits 16,32 >> gpurun_out/r02c_wgrad.json
timeout -k 10 120 python tools/wgrad_bench.py --splits 4,8 >> gpurun_out/r02c_wgrad.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/r02c_pmc -o run -- python tools/wgrad_bench.py --reps 10 > gpurun_out/r02c_pmc.log 2>&1
