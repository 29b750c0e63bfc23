# A/B of an environment knob on the bench (one GPU call): bash tools/gpu_ab_env.sh OUT VAR v1 v2 ...
# each value runs the short bench twice (interleaved rounds); one line per run in OUT
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$1; VAR=$2; shift 2
for round in 1 2; do
  for v in "$@"; do
    r=$(env "$VAR=$v" timeout -k 10 120 python bench.py --steps 100 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 300 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
k = d['kernels']
print(json.dumps({'value': round(d['value']), 'long': round(d['timed_long']['value']),
      'ms_long': round(d['timed_long']['ms_per_step'], 4),
      'us': {n: k[n]['avg_us'] for n in k}}))")
    echo "$VAR=$v round=$round $r" >> "$OUT"
  done
done
