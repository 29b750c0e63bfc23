#!/bin/bash
# One gpurun call of round 6 (run from the repo root through gpurun): the named steps in order,
# each under its own time limit; a fault / abort / timeout (exit status other than 0 or 1) ends
# the call there. Output under gpurun_out/TAG/.
#   tests     GPU test suite
#   mlptests  the MLP / learner GPU tests only
#   smoke     __graft_entry__.smoke()
#   wgrad     tools/wgrad_bench.py on this tree's library
#   abprev    interleaved same-box bench A/B (3 rounds): this tree vs abl/prev (a copy of the
#             previous round's tree with its own built library; removed before the round ends)
#   bench     the default bench line
#   prof      rocprofv3 kernel trace + stats of a short bench
#   pmc       FETCH_SIZE / WRITE_SIZE / SQ passes of a short bench (separate runs)
#   vab       interleaved bench A/B (3 rounds, kernel times included): this tree's library vs
#             each abl/libnavenv_$v.so named in $VARS (bound through tools/withlib.py; `prev` =
#             the previous HEAD's library, tools/build_prev.sh)
#   clock     held shader clock of the row kernels (tools/clock_probe.py on abl/libnavenv_clock.so)
#   sphost    tools/shared_policy_host.py: config 5's learner host cost at rank batch 4 096
#   shape     tools/probe/mfma_shape_probe (build/mfma_shape_probe): 32x32x16 vs 16x16x32 split GEMM
#   phase     critic_rows phase trace (abl/libnavenv_$v.so for each $v in $PVARS, default
#             trace) at batch 32768 (two workgroups per CU) and 16448 (one), and act_tick's
#   wpmc      SQ counters and timing of tools/wgrad_bench.py for this tree's library and each
#             abl/libnavenv_$v.so named in $WVARS (A/B variants built by tools/build_variant.sh)
#   launch    bench.py --gpus 2 without an outer torch.distributed.run (the launcher path), as a
#             one-box rehearsal (NAV_DIST_REHEARSAL=1: both ranks on cuda:0, gloo): independent
#             blocks, shared policy, shared policy + overlapped collect
# usage: bash tools/gpu_r06.sh TAG step...
set -u
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
: > "$O/status.txt"
SHORT="--steps 20 --warmup 3 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0"
PMCB="--steps 4 --warmup 2 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0"
run() {
  local name=$1 t=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$O/status.txt"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    tests) run gputest 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    alltests) run gputest_all 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    acc) run accuracy 300 python -u -m pytest tests/test_gpu_mlp.py -m gpu -k "split_gemm_f32_accuracy or gradients_vs_reference or weight_grads_2layer" -v -s --timeout 120 --timeout-method thread ;;
    sptests) run sptest 400 python -u -m pytest tests/test_gpu_shared_policy.py tests/test_gpu_checkpoint.py -m gpu -x -v --timeout 240 --timeout-method thread ;;
    dbgw) run dbg_wgrad 200 python tools/dbg_wgrad.py ;;
    mlptests) run mlptest 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    wgrad) run wgrad 200 python tools/wgrad_bench.py ;;
    wgscan) run wg_32768 120 python tools/wgrad_bench.py &&
            run wg_16384 120 python tools/wgrad_bench.py --batch 16384 &&
            run wg_65536 120 python tools/wgrad_bench.py --batch 65536 &&
            run wg_s8 120 python tools/wgrad_bench.py --splits 8,8 &&
            run wg_s32 120 python tools/wgrad_bench.py --splits 32,32 ;;
    abprev) for r in 1 2 3; do
          run ab_new_$r 200 python bench.py $SHORT --steps 100 --warmup 10 --no-timed-events
          (cd abl/prev && run ab_old_$r 200 python bench.py $SHORT --steps 100 --warmup 10 --no-timed-events)
        done ;;
    bench) run bench 500 python bench.py ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python bench.py $SHORT ;;
    pmc) run pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python bench.py $PMCB &&
         run pmc_write 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python bench.py $PMCB &&
         run pmc_sq 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/sq" -o run -- python bench.py $PMCB ;;
    wpmc) for v in "" $WVARS; do
            tag=${v:-base}
            W=(); [ -n "$v" ] && W=(tools/withlib.py "$ROOT/abl/libnavenv_$v.so")
            run wpmc_$tag 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/wpmc_$tag" -o run -- python "${W[@]}" tools/wgrad_bench.py --reps 5
            run wvar_$tag 120 python "${W[@]}" tools/wgrad_bench.py
          done ;;
    vab) for r in 1 2 3; do
           for v in "" $VARS; do
             tag=${v:-base}
             W=(); [ -n "$v" ] && W=(tools/withlib.py "$ROOT/abl/libnavenv_$v.so")
             run vab_${tag}_$r 200 python "${W[@]}" bench.py $SHORT --steps 60 --warmup 5
           done
         done ;;
    phase) for v in ${PVARS:-trace}; do
             W=(tools/withlib.py "$ROOT/abl/libnavenv_$v.so")
             run phase_${v}_32768 200 python "${W[@]}" tools/phase_trace.py --batch 32768
             run phase_${v}_16448 200 python "${W[@]}" tools/phase_trace.py --batch 16448
             run phase_${v}_tick 200 python "${W[@]}" tools/phase_trace.py --tick
           done ;;
    phase1) for v in ${PV1:-trace7}; do
              W=(tools/withlib.py "$ROOT/abl/libnavenv_$v.so")
              run phase1_$v 200 python "${W[@]}" tools/phase_trace.py --batch 100 --hidden 200 --n-hidden 3 --n-envs 1024
            done ;;
    wtrace1) run wtrace1 200 python tools/withlib.py "$ROOT/abl/libnavenv_wtrace.so" tools/wgrad_trace.py --batch 100 --hidden 200 --n-hidden 3 --n-envs 1024 ;;
    wtrace) for v in ${TVARS:-wtrace}; do
              run ${v}_32k 200 python tools/withlib.py "$ROOT/abl/libnavenv_$v.so" tools/wgrad_trace.py &&
              run ${v}_16k 200 python tools/withlib.py "$ROOT/abl/libnavenv_$v.so" tools/wgrad_trace.py --batch 16384
            done ;;
    clock) run clock 200 python tools/withlib.py "$ROOT/abl/libnavenv_clock.so" tools/clock_probe.py --seconds 3 ;;
    sphost) run sphost 300 python tools/shared_policy_host.py ;;
    launch) export NAV_DIST_REHEARSAL=1
            run launch_blocks 300 python bench.py --gpus 2 --steps 20 --warmup 2 --long-steps 0 &&
            run launch_shared 300 python bench.py --gpus 2 --steps 20 --warmup 2 --long-steps 0 --shared-policy &&
            run launch_overlap 300 python bench.py --gpus 2 --steps 20 --warmup 2 --long-steps 0 --shared-policy --overlap-collect
            unset NAV_DIST_REHEARSAL ;;
    dbgvar) for v in $DVARS; do run dbg_$v 120 python tools/withlib.py "$ROOT/abl/libnavenv_$v.so" tools/dbg_bits.py --batch 16421; done ;;
    dbgbits) run dbgbits_16421 120 python tools/dbg_bits.py --batch 16421 &&
             run dbgbits_2048 120 python tools/dbg_bits.py --batch 2048 ;;
    wgab) for r in 1 2 3; do for v in "" $WVARS; do tag=${v:-base}
            W=(); [ -n "$v" ] && W=(tools/withlib.py "$ROOT/abl/libnavenv_$v.so")
            run wgab_${tag}_$r 120 python "${W[@]}" tools/wgrad_bench.py; done; done ;;
    c1prof) run c1prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c1trace" -o run -- python tools/config1_run.py
            rm -f "$O/c1trace/run_kernel_trace.csv" ;;  # ~100 k rows: over gpurun's copy-back cap
    config1) run config1 300 python tools/config1_run.py ;;
    mix) run mix 100 ./build/mix_probe ;;
    shape) run shape 200 ./build/mfma_shape_probe 512 2.5 0 && run shape_dz 200 ./build/mfma_shape_probe 512 2.5 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done >> "$O/status.txt"
