# Round 6, call AG: split-K sum with every partial's load issued first (SPLITK_SUM_BATCH=1, HEAD)
# against the one-at-a-time loop (abv/sk0) -- FP6 / config tests, config-3 graph steps interleaved,
# kernel stats of HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp6.py tests/test_gpu_net_configs.py tests/test_gpu_graph.py \
  > gpurun_out/r06_ag_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_ag_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_ag_gpu_tests.log | tail -1
for rep in 1 2 3; do
  for lib in head sk0; do
    if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
    tag=mlpg_${lib}_$rep
    timeout -k 10 300 python bench.py --config mlp --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ag_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_ag_$tag.log; exit 1; }
    echo "$tag: $(tail -1 gpurun_out/r06_ag_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
unset BNN_LIB
cd /tmp && export TMPDIR=/tmp
for lib in head sk0; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06ag_$lib -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_ag_prof_$lib.log 2>&1 || { echo PROF FAIL; exit 1; }
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06ag_$lib -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_ag_mlpg_stats_$lib.txt
  echo "== $lib"; grep -E "kernel time|splitk" $R/gpurun_out/r06_ag_mlpg_stats_$lib.txt | cut -c1-120
done
