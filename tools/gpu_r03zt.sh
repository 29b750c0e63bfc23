# One GPU call: GPU suite, then the small-batch forms A/B: config 1's drop-in td3_update (3x200,
# batch 100: 32-row blocks, NT 7) vs abl/libnavenv_sb1.so, and the bench at batch 8 192 (32-row
# blocks, NT 8) vs abl/libnavenv_sb1_8.so (both: one stage buffer, two barriers per step).
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
for r in 1 2; do
  for v in "NAV_X=0" "NAV_LIB=abl/libnavenv_sb1.so"; do
    echo "[$v] $(env $v timeout -k 10 300 python tools/prof_td3_host.py 1000 2>/dev/null | grep 'ms per update')" >> $O/c1_ab.log
  done
  for v in "NAV_X=0" "NAV_LIB=abl/libnavenv_sb1_8.so"; do
    echo "[$v] $(env $v timeout -k 10 200 python bench.py --batch 8192 --steps 40 --warmup 5 --no-timed-events 2>/dev/null | tail -1)" >> $O/utd025_ab.log
  done
done
timeout -k 10 300 python tools/config1_run.py > $O/config1_run.json 2> $O/config1_run.err
echo done > $O/DONE
