# Round 6, call J: coalesced Adam pass of the 64 x 64 pack tiles + the elementwise cross-entropy
# backward / prefetching forward -- the tests that cover them, then interleaved small-config benches
# against the previous commit's library (abv/pre6829).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_graph.py \
  tests/test_gpu_loss.py tests/test_gpu_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py tests/test_gpu_pixels.py \
  > gpurun_out/r06_j_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_j_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_j_gpu_tests.log | tail -1
for rep in 1 2; do
  for lib in head pre; do
    if [ $lib = pre ]; then export BNN_LIB=$R/abv/pre6829/libbnn.so; else unset BNN_LIB; fi
    for c in "mlp --graph" "small --graph" "cnn --graph"; do
      tag=$(echo $c | tr -d ' -')_${lib}_$rep
      timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_j_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_j_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_j_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
