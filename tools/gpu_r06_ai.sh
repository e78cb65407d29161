# Round 6, call AI: the fused head's statistics chunks at >= 32 rows (abv/hm32) against 16 (HEAD) --
# head tests on that build, config-3 graph steps interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BNN_LIB=$R/abv/hm32/libbnn.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_head.py tests/test_gpu_net_configs.py \
  > gpurun_out/r06_ai_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_ai_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_ai_gpu_tests.log | tail -1
for rep in 1 2 3; do
  for lib in head hm32; do
    if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
    tag=mlpg_${lib}_$rep
    timeout -k 10 300 python bench.py --config mlp --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ai_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_ai_$tag.log; exit 1; }
    echo "$tag: $(tail -1 gpurun_out/r06_ai_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
