# Round 6, call U: BatchNorm final merges with 16 / 4 / 1 columns per workgroup by layer width
# (narrow layers: more workgroups, fewer partials per thread) -- the GPU suite part A, then
# interleaved small-config graph steps and the wide step against the previous build (abv/preffin).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_u_gpu_tests_a.log 2>&1 || { echo SUITE A FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_u_gpu_tests_a.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_u_gpu_tests_a.log | tail -1
for rep in 1 2; do
  for lib in pre head; do
    if [ $lib = pre ]; then export BNN_LIB=$R/abv/preffin/libbnn.so; else unset BNN_LIB; fi
    for c in "mlp --graph" "cnn --graph" "small --graph"; do
      tag=$(echo $c | tr -d ' -')_${lib}_$rep
      timeout -k 10 300 python bench.py --config $c --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_u_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_u_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_u_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
