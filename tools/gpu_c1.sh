# One GPU call: config 1 end to end and the drop-in td3_update profile. usage: bash tools/gpu_c1.sh TAG
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python tools/config1_run.py > $O/config1_run.json 2> $O/config1_run.err
timeout -k 10 300 python tools/prof_td3_host.py 5000 > $O/td3_host_5000.log 2>&1
timeout -k 10 300 python tools/prof_td3_host.py 1000 > $O/td3_host_1000.log 2>&1
echo done > $O/DONE
