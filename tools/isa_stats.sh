#!/bin/bash
# Compile a .hip file to gfx950 assembly and print per-kernel register / scratch / instruction
# counts for kernels whose mangled name matches $2 (grep -E pattern).
# usage: tools/isa_stats.sh residual-td3-robot-navigation_amd/csrc/mlp_kernels.hip 'k_mlp_fwdILi8ELi2'
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1
PAT=${2:-.}
OUT=${ISA_OUT:-/tmp/isa_$(basename "$SRC" .hip).s}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$ROOT/include" \
  -I"$ROOT/residual-td3-robot-navigation_amd/csrc" --cuda-device-only -S -o "$OUT" "$SRC" 2>/dev/null
awk -v pat="$PAT" '
  /^_Z[^ ]*:/ { name = $1; sub(":", "", name); on = (name ~ pat); n_mfma = n_flat = n_exec = n_scr = n_bar = n_ds = n_gl = 0; next }
  on && /v_mfma/ { n_mfma++ }
  on && /flat_load|flat_store/ { n_flat++ }
  on && /saveexec/ { n_exec++ }
  on && /scratch_/ { n_scr++ }
  on && /s_barrier/ { n_bar++ }
  on && /ds_read|ds_write/ { n_ds++ }
  on && /global_load|global_store|buffer_load|buffer_store/ { n_gl++ }
  on && /; NumVgprs:/ { vg = $3 }
  on && /; NumAgprs:/ { ag = $3 }
  on && /; ScratchSize:/ { printf "%-60s vgpr %s agpr %s scratch %s mfma %d ds %d global %d flat %d saveexec %d scratch_ops %d barriers %d\n", substr(name, 1, 60), vg, ag, $3, n_mfma, n_ds, n_gl, n_flat, n_exec, n_scr, n_bar; on = 0 }
' "$OUT"
