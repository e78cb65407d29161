# Keep-bit plane (LDS-staged words in the q6 pass, per-call q6 store addresses: no spills) and the
# 2-column head statistics pass: parity tests, then wide-step A/B with kernel-trace stats:
#   kb1_c4 (keep bits, 4 columns), kb1_c2 (keep bits, 2 columns), kb0_c4 (hash, 4 columns)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_keep_bits.py tests/test_gpu_z16.py tests/test_gpu_q6_handoff.py tests/test_gpu_head.py tests/test_gpu_wide_step.py > gpurun_out/r05_kb2_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/r05_kb2_tests.log; exit 1; }
tail -2 gpurun_out/r05_kb2_tests.log
cd /tmp && export TMPDIR=/tmp
for cfg in "1 4" "1 2" "0 4"; do
  set -- $cfg
  tag=kb$1_c$2
  rm -rf $R/gpurun_out/kb2_prof_$tag
  BNN_KEEP_BITS=$1 BNN_HEAD_RED_COLS=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kb2_prof_$tag -o wide --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r05_kb2_bench_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -20 $R/gpurun_out/r05_kb2_bench_$tag.log; exit 1; }
  echo "$tag $(tail -1 $R/gpurun_out/r05_kb2_bench_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  python3 $R/tools/prof_summary.py $(find $R/gpurun_out/kb2_prof_$tag -name 'wide_kernel_stats.csv' | head -1) 13 40 | grep -E "step|head|q6_k|reduce_k<0|keep|dz_quant" | cut -c1-150
done
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_kb2_bench_plain.log 2>&1 && tail -1 gpurun_out/r05_kb2_bench_plain.log | cut -c1-200
