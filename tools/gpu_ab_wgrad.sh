set -e
cd $GRAFT_REPO_ROOT
for lib in residual-td3-robot-navigation_amd/nav/libnavenv.so abl/libnavenv_exp1.so abl/libnavenv_exp2.so abl/libnavenv_w4.so; do
  echo "$lib $(NAV_LIB=$lib timeout -k 10 120 python tools/wgrad_bench.py)" >> gpurun_out/r02f_ab.log
done
