# Round 6, call Y: the fused head's backward statistics on chunks of >= 16 rows (config 3: 1,024 ->
# 256 chunk partials, keep bits read instead of re-hashed) -- head / config tests, then interleaved
# config-3 graph steps against the previous build (abv/prehead) and kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_head.py \
  tests/test_gpu_net_configs.py tests/test_gpu_graph.py tests/test_gpu_training.py tests/test_gpu_keep_bits.py \
  tests/test_gpu_z16.py tests/test_gpu_q6_handoff.py tests/test_gpu_rccl.py \
  > gpurun_out/r06_y_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_y_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_y_gpu_tests.log | tail -1
for rep in 1 2 3; do
  for lib in pre head; do
    if [ $lib = pre ]; then export BNN_LIB=$R/abv/prehead/libbnn.so; else unset BNN_LIB; fi
    tag=mlpgraph_${lib}_$rep
    timeout -k 10 300 python bench.py --config mlp --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_y_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_y_$tag.log; exit 1; }
    echo "$tag: $(tail -1 gpurun_out/r06_y_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
unset BNN_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06y_mlpg -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_y_mlpg_prof.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_y_mlpg_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06y_mlpg -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_y_mlpg_stats.txt
grep -E "kernel time|head|bwd_final|keep_bits" $R/gpurun_out/r06_y_mlpg_stats.txt | cut -c1-140
