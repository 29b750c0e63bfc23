# One GPU call: the GPU suite, then config 1 end to end (tools/config1_run.py) and the drop-in
# td3_update host/device profile (tools/prof_td3_host.py). usage: bash tools/gpu_config1.sh TAG
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 300 python tools/config1_run.py > $O/config1_run.json 2> $O/config1_run.err
timeout -k 10 300 python tools/prof_td3_host.py 5000 > $O/td3_host_5000.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c1trace -o run -- python tools/prof_td3_host.py 1000 > $O/c1trace.log 2>&1
echo done > $O/DONE
