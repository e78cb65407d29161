# Round 6, call AH: the int8 column quantiser on 2 row tiles per workgroup for small grids
# (QC_RT_SMALL=2, HEAD) against 8 (abv/qc8) -- pixel / config / training tests on HEAD, config-3 graph
# steps interleaved, kernel stats of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pixels.py tests/test_gpu_s20.py \
  tests/test_gpu_net_configs.py tests/test_gpu_training.py tests/test_gpu_graph.py tests/test_gpu_parity.py \
  > gpurun_out/r06_ah_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_ah_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_ah_gpu_tests.log | tail -1
for rep in 1 2 3; do
  for lib in head qc8; do
    if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
    tag=mlpg_${lib}_$rep
    timeout -k 10 300 python bench.py --config mlp --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ah_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_ah_$tag.log; exit 1; }
    echo "$tag: $(tail -1 gpurun_out/r06_ah_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
unset BNN_LIB
cd /tmp && export TMPDIR=/tmp
for lib in head qc8; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06ah_$lib -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_ah_prof_$lib.log 2>&1 || { echo PROF FAIL; exit 1; }
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06ah_$lib -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_ah_mlpg_stats_$lib.txt
  echo "== $lib"; grep -E "kernel time|quant_cols|dz_colsum" $R/gpurun_out/r06_ah_mlpg_stats_$lib.txt | cut -c1-120
done
