# wgrad microbench A/B over variant libraries (tuning only): usage bash tools/gpu_ab_wgrad.sh OUT lib...
set -e
cd $GRAFT_REPO_ROOT
out=$1; shift
for lib in "$@"; do
  echo "$lib $(NAV_LIB=$lib timeout -k 10 120 python tools/wgrad_bench.py)" >> "$out"
done
