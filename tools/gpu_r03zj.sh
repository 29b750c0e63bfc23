# One GPU call: GPU suite, bench A/B with kernel traces (this tree vs abl/ libraries), config 1's
# drop-in td3_update A/B. usage: bash tools/gpu_r03zj.sh TAG libs...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
bash tools/gpu_ab_libs_trace.sh "$@"
shift
for r in 1 2; do
  for v in "NAV_X=0" "${@/#/NAV_LIB=}"; do
    echo "[$v] $(env $v timeout -k 10 300 python tools/prof_td3_host.py 5000 2>/dev/null | grep 'ms per update')" >> $O/c1_ab.log
  done
done
echo done > $O/DONE_ALL
