# One GPU call: GPU suite, library A/B with kernel traces (this tree vs abl/ variants), config 1
# end to end and the drop-in td3_update host profile. usage: bash tools/gpu_r03zf.sh TAG libs...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
bash tools/gpu_ab_libs_trace.sh "$@"
timeout -k 10 300 python tools/config1_run.py > $O/config1_run.json 2> $O/config1_run.err
timeout -k 10 300 python tools/prof_td3_host.py 5000 > $O/td3_host_5000.log 2>&1
echo done > $O/DONE_ALL
