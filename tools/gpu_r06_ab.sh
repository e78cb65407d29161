# Round 6, call AB: FP6 half tiles on small unsplit grids (abv/hsmall, FP6_HALF_SMALL=1) -- the FP6 and
# config tests on that build, then config 3 / BinCNN graph steps interleaved with HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BNN_LIB=$R/abv/hsmall/libbnn.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp6.py tests/test_gpu_net_configs.py \
  > gpurun_out/r06_ab_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_ab_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_ab_gpu_tests.log | tail -1
for rep in 1 2 3; do
  for cfg in mlp; do
    for lib in head hsmall; do
      if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
      tag=${cfg}g_${lib}_$rep
      timeout -k 10 300 python bench.py --config $cfg --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ab_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_ab_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_ab_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
unset BNN_LIB
for lib in head hsmall; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 python bench.py --config cnn --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ab_cnng_$lib.log 2>&1 || exit 1
  echo "cnng_$lib: $(tail -1 gpurun_out/r06_ab_cnng_$lib.log | grep -o '"ms_per_step": [0-9.]*')"
done
