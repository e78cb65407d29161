# Round 6, call Q: the backward-data conv kernel with a scalar tap loop (Cop = 32) -- the BinCNN tests,
# then
# interleaved BinCNN eager / graph timings against the previous build (abv/preconv) and kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cnn_parity.py \
  tests/test_gpu_parity.py tests/test_gpu_conv_popc.py tests/test_gpu_parallel.py tests/test_gpu_rccl.py tests/test_gpu_training.py \
  > gpurun_out/r06_q_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_q_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_q_gpu_tests.log | tail -1
for rep in 1 2; do
  for lib in head pre; do
    if [ $lib = pre ]; then export BNN_LIB=$R/abv/preconv/libbnn.so; else unset BNN_LIB; fi
    for c in "cnn" "cnn --graph"; do
      tag=$(echo $c | tr -d ' -')_${lib}_$rep
      timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_q_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_q_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_q_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
unset BNN_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06m_cnng -o cnng --output-format csv -- python3 $R/bench.py --config cnn --graph --steps 100 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_q_cnng_prof.log 2>&1 || { echo PROF CNNG FAIL; tail -5 $R/gpurun_out/r06_q_cnng_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06m_cnng -name 'cnng_kernel_stats.csv' | head -1) 105 40 > $R/gpurun_out/r06_q_cnng_stats.txt
head -16 $R/gpurun_out/r06_q_cnng_stats.txt | cut -c1-150
