# Dropout keep-bit plane: parity tests, then the wide step A/B (BNN_KEEP_BITS=1 default vs 0) with
# per-kernel timings of the head passes (rocprofv3 kernel-trace stats).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_keep_bits.py tests/test_gpu_z16.py tests/test_gpu_q6_handoff.py tests/test_gpu_head.py > gpurun_out/r05_kb_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/r05_kb_tests.log; exit 1; }
tail -2 gpurun_out/r05_kb_tests.log
cd /tmp && export TMPDIR=/tmp
for kb in 1 0; do
  rm -rf $R/gpurun_out/kb_prof_$kb
  BNN_KEEP_BITS=$kb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kb_prof_$kb -o wide --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r05_kb_bench_$kb.log 2>&1 || { echo BENCH $kb FAIL; tail -20 $R/gpurun_out/r05_kb_bench_$kb.log; exit 1; }
  echo "keep_bits=$kb $(tail -1 $R/gpurun_out/r05_kb_bench_$kb.log | grep -o '"ms_per_step": [0-9.]*')"
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/kb_prof_$kb -name 'wide_kernel_stats.csv' | head -1) 13 12 | cut -c1-150
done
