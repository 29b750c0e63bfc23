set -e
cd $GRAFT_REPO_ROOT
for lib in residual-td3-robot-navigation_amd/nav/libnavenv.so abl/libnavenv_exp4.so abl/libnavenv_exp5.so; do
  echo "$lib $(NAV_LIB=$lib timeout -k 10 120 python tools/wgrad_bench.py)" >> gpurun_out/r02n_ab.log
done
