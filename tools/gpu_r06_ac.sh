# Round 6, call AC: the 256 x 256 BatchNorm apply-pack on config 3's small layers (abv/apf32,
# AP_FAST_MIN_TILES=32) against HEAD -- graph steps interleaved, then per-kernel stats of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in head apf32; do
    if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
    tag=mlpg_${lib}_$rep
    timeout -k 10 300 python bench.py --config mlp --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ac_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_ac_$tag.log; exit 1; }
    echo "$tag: $(tail -1 gpurun_out/r06_ac_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in head apf32; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06ac_$lib -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_ac_prof_$lib.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_ac_prof_$lib.log; exit 1; }
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06ac_$lib -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_ac_mlpg_stats_$lib.txt
  echo "== $lib"; grep -E "kernel time|pack" $R/gpurun_out/r06_ac_mlpg_stats_$lib.txt | cut -c1-120
done
