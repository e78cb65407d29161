# Round 6, call Z: BatchNorm chunk fill threshold A/B (BN_FILL_LOG2 17 = HEAD, 16, 15 via abv/fill*),
# config 3 and BinCNN graph steps interleaved, then per-kernel stats of the config-3 variants.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in mlp cnn; do
    for lib in head fill16 fill15; do
      if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
      tag=${cfg}g_${lib}_$rep
      timeout -k 10 300 python bench.py --config $cfg --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_z_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_z_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_z_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in head fill16; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06z_$lib -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_z_prof_$lib.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_z_prof_$lib.log; exit 1; }
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06z_$lib -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_z_mlpg_stats_$lib.txt
  echo "== $lib"; grep -E "kernel time|bn_|q6" $R/gpurun_out/r06_z_mlpg_stats_$lib.txt | cut -c1-120
done
