# One GPU call: the forward kernel's 64-row double-buffered stage (abl/libnavenv_db2.so): its
# forward / fused-tick GPU tests, then the bench A/B with kernel traces.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
NAV_LIB=abl/libnavenv_db2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest_db2.log 2>&1
bash tools/gpu_ab_libs_trace.sh $1 abl/libnavenv_db2.so
echo done > $O/DONE_ALL
