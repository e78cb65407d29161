# Round 6, call AA: FP6 split-K cap A/B (FP6_SPLIT_CAP 1024 = HEAD, 1 / 2 / 4 / 8 via abv/cap*), config 3,
# BinCNN and the small net as graphs, interleaved, then per-kernel stats of HEAD and cap 4 on config 3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in mlp cnn small; do
    for lib in head cap1 cap2 cap4 cap8; do
      if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
      tag=${cfg}g_${lib}_$rep
      timeout -k 10 300 python bench.py --config $cfg --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_aa_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_aa_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_aa_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in head cap4 cap2; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06aa_$lib -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_aa_prof_$lib.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_aa_prof_$lib.log; exit 1; }
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06aa_$lib -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_aa_mlpg_stats_$lib.txt
  echo "== $lib"; grep -E "kernel time|fp6|splitk" $R/gpurun_out/r06_aa_mlpg_stats_$lib.txt | cut -c1-120
done
