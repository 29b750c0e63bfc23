#!/bin/bash
# A/B variant of the row kernels at hidden width 256 (tuning only): the dispatch object (part 0)
# and the NT = 8 row kernels rebuilt with extra -D flags, linked with the tree's other objects.
#   tools/build_rows_variant.sh NAME "-DFOO=1 ..."  -> abl/libnavenv_NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2
P=residual-td3-robot-navigation_amd
B=$P/build
make -s -C $P
mkdir -p abl
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -I$P/csrc -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp"
/opt/rocm/bin/hipcc $FL $flags -DNAV_MLP_PART=0 -c $P/csrc/mlp_kernels.hip -o abl/${name}_p0.o &
/opt/rocm/bin/hipcc $FL $flags -DNAV_MLP_PART=8 -c $P/csrc/mlp_kernels.hip -o abl/${name}_p8.o &
wait
objs="$B/env_kernels.o $B/learner_kernels.o abl/${name}_p0.o abl/${name}_p8.o"
for n in 1 2 3 4 5 6 7; do objs="$objs $B/mlp_nt$n.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libnavenv_$name.so $objs
echo abl/libnavenv_$name.so
