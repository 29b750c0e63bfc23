# One GPU call: row-kernel library A/B with traces (tools/gpu_ab_libs_trace.sh), then config 1 end
# to end with the weight-gradient step fused / unfused.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_ab_libs_trace.sh "$@"
O=gpurun_out/$1
for f in 0 1; do
  NAV_FUSE_WGRAD_STEP=$f timeout -k 10 300 python tools/config1_run.py > $O/config1_fuse$f.json 2> $O/config1_fuse$f.err
done
echo done > $O/DONE_ALL
