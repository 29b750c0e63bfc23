# One GPU call: GPU suite, then the library A/B with kernel traces. usage: bash tools/gpu_r03zq.sh TAG libs...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
bash tools/gpu_ab_libs_trace.sh "$@"
echo done > $O/DONE_ALL
