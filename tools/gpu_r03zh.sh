# One GPU call: GPU suite, library A/B with kernel traces, and a kernel trace of the drop-in
# td3_update (config 1's learner) at 1000 replay rows. usage: bash tools/gpu_r03zh.sh TAG libs...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
bash tools/gpu_ab_libs_trace.sh "$@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c1trace -o run -- python tools/prof_td3_host.py 1000 > $O/c1trace.log 2>&1
echo done > $O/DONE_ALL
