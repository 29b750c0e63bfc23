# One GPU call: GPU suite, kernel trace of the default bench, A/B of the row kernels (HEAD~ mlp8
# object vs this tree), phase trace of critic_rows.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > $O/trace.log 2>&1
rm -f gpurun_out/ab.log
timeout -k 10 900 bash tools/ab.sh 3 "NAV_LIB=abl/libnavenv_oldmlp.so" "NAV_FUSE_WGRAD_STEP=0" > $O/ab.txt 2>&1
cp gpurun_out/ab.log $O/ab.log
NAV_LIB=abl/libnavenv_trace.so timeout -k 10 300 python tools/phase_trace.py > $O/phase_trace.json 2> $O/phase_trace.err
echo done > $O/DONE
