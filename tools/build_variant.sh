#!/bin/bash
# Build an A/B variant of libnavenv.so with extra -D flags on one translation unit (tuning only):
#   tools/build_variant.sh NAME learner|env|mlpN "-DFOO=1 ..."  (mlpN: the row kernels of hidden
#   width 32*N; mlp8 = 256; mlp0 = the row kernels' C-ABI object)
# -> abl/libnavenv_NAME.so (bind it with python tools/withlib.py abl/libnavenv_NAME.so SCRIPT ...)
set -eu
cd "$(dirname "$0")/.."
name=$1; unit=$2; flags=$3
P=residual-td3-robot-navigation_amd
B=$P/build
make -s -C $P
mkdir -p abl
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -I$P/csrc"
objs="$B/env_kernels.o $B/learner_kernels.o $B/mlp_kernels.o"
for n in 1 2 3 4 5 6 7 8; do objs="$objs $B/mlp_nt$n.o"; done
case $unit in
  learner) sched="-mllvm -amdgpu-sched-strategy=max-ilp"
           [ -n "${NOSCHED:-}" ] && sched=""  # NOSCHED=1: the default machine scheduler
           /opt/rocm/bin/hipcc $FL $sched $flags -c $P/csrc/learner_kernels.hip -o abl/$name.o
           objs=${objs/$B\/learner_kernels.o/abl\/$name.o} ;;
  env) /opt/rocm/bin/hipcc $FL $flags -c $P/csrc/env_kernels.hip -o abl/$name.o
       objs=${objs/$B\/env_kernels.o/abl\/$name.o} ;;
  mlp0) /opt/rocm/bin/hipcc $FL -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp -fno-slp-vectorize $flags -DNAV_MLP_PART=0 -c $P/csrc/mlp_kernels.hip -o abl/$name.o
        objs=${objs/$B\/mlp_kernels.o/abl\/$name.o} ;;
  mlp[1-8]) n=${unit#mlp}
        /opt/rocm/bin/hipcc $FL -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp -fno-slp-vectorize $flags -DNAV_MLP_PART=$n -c $P/csrc/mlp_kernels.hip -o abl/$name.o
        objs=${objs/$B\/mlp_nt$n.o/abl\/$name.o} ;;
  mlp8agpr) /opt/rocm/bin/hipcc $FL $flags -DNAV_MLP_PART=8 -c $P/csrc/mlp_kernels.hip -o abl/$name.o
        objs=${objs/$B\/mlp_nt8.o/abl\/$name.o} ;;
  *) echo "unit?"; exit 2 ;;
esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libnavenv_$name.so $objs
echo abl/libnavenv_$name.so
