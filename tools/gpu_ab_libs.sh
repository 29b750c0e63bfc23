# A/B of library variants (one GPU call): bash tools/gpu_ab_libs.sh OUT "cmd args" lib1 lib2 ...
# runs `NAV_LIB=<lib> cmd` for each library, two interleaved rounds, one line per run in OUT
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$1; CMD=$2; shift 2
for round in 1 2; do
  for lib in "$@"; do
    echo "$lib round=$round $(NAV_LIB=$lib timeout -k 10 120 $CMD)" >> "$OUT"
  done
done
