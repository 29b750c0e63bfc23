# One GPU call: config 1's drop-in td3_update (replay 1000) with the weight-gradient step fused
# (NAV_FUSE_WGRAD_STEP=1) or not, interleaved. usage: bash tools/gpu_c1_fuse_ab.sh TAG
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; mkdir -p $O
for r in 1 2 3; do
  for f in 0 1; do
    echo "[NAV_FUSE_WGRAD_STEP=$f] $(NAV_FUSE_WGRAD_STEP=$f timeout -k 10 300 python tools/prof_td3_host.py 1000 2>/dev/null | grep 'ms per update')" >> $O/c1_fuse_ab.log
  done
done
echo done > $O/DONE
