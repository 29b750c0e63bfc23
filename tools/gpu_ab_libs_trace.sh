# One GPU call: for each library (this tree's and abl/ variants given as arguments), a kernel
# trace of a short bench, then a 2-round interleaved A/B of the bench step.
# usage: bash tools/gpu_ab_libs_trace.sh TAG abl/libnavenv_x.so ...
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/$1; shift; mkdir -p $O
i=0
for lib in default "$@"; do
  if [ "$lib" = default ]; then e=""; else e="NAV_LIB=$lib"; fi
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace$i -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-utd-sweep --no-sweep --long-steps 0 > $O/trace$i.log 2>&1
  echo "$i $lib" >> $O/traces.txt
  i=$((i+1))
done
rm -f gpurun_out/ab.log
args=("NAV_X=0")
for lib in "$@"; do args+=("NAV_LIB=$lib"); done
timeout -k 10 900 bash tools/ab.sh 2 "${args[@]}" > $O/ab.txt 2>&1
cp gpurun_out/ab.log $O/ab.log
echo done > $O/DONE
