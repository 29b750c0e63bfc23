# One GPU call: the step-kernel sweep point at 2^24 envs (bench.py --sweep-only), this tree vs the
# abl/ libraries given, interleaved x3. usage: bash tools/gpu_sweep_ab.sh TAG libs...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2 3; do
  for v in "NAV_X=0" "${@/#/NAV_LIB=}"; do
    echo "[$v] $(env $v timeout -k 10 200 python bench.py --sweep-only 16777216 2>/dev/null | tail -1)" >> $O/sweep_ab.log
  done
done
echo done > $O/DONE
