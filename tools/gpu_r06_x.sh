# Round 6, call X: the fused head's bias gradient on one libbnn launch (bnn_col_sums_narrow) instead
# of torch's reduction -- tests, then interleaved config-3 / small / wide-MLP graph steps against
# the previous build (abv/precs; the Python side is HEAD's in both, the old build lacks the symbol
# only if it is called, so the A/B sets BNN_COLSUM=0 for it).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_head.py \
  tests/test_gpu_net_configs.py tests/test_gpu_graph.py tests/test_gpu_training.py tests/test_gpu_parity.py \
  > gpurun_out/r06_x_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_x_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_x_gpu_tests.log | tail -1
for rep in 1 2 3; do
  for v in 0 1; do
    for c in "mlp --graph" "small --graph"; do
      tag=$(echo $c | tr -d ' -')_cs${v}_$rep
      BNN_COLSUM=$v timeout -k 10 300 python bench.py --config $c --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_x_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_x_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_x_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
