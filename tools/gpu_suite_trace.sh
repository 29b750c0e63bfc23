# One GPU call: the GPU suite, then a rocprofv3 kernel trace + stats of a short bench (set-up
# kernels included). usage: bash tools/gpu_suite_trace.sh TAG
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > $O/trace.log 2>&1
echo done > $O/DONE
