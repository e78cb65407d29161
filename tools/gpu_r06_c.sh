# Round 6, call C: the half-tile FP6 dX default, the drop-in's pixel recognition and fused sign
# write-back: the GPU suite (part A, then the long tests), smoke, bench, drop-in kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_c_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_c_gpu_tests_a.log | tail -2; grep -E "^FAILED|Error" gpurun_out/r06_c_gpu_tests_a.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/r06_c_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r06_c_gpu_tests_b.log | tail -2; grep -E "^FAILED|Error" gpurun_out/r06_c_gpu_tests_b.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06_c_smoke.log 2>&1 || { echo SMOKE FAIL; tail -5 gpurun_out/r06_c_smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r06_c_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r06_c_bench.log; exit 1; }
tail -1 gpurun_out/r06_c_bench.log | cut -c1-200; tail -1 gpurun_out/r06_c_bench.log | grep -o '"dropin": {[^}]*}'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06c_dropin -o run --output-format csv -- python3 $R/bench.py --dropin --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_c_dropin_prof.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/r06_c_dropin_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06c_dropin -name 'run_kernel_stats.csv' | head -1) 7 40 > $R/gpurun_out/r06_c_dropin_stats.txt
head -24 $R/gpurun_out/r06_c_dropin_stats.txt | cut -c1-170
cd $R
timeout -k 10 300 python -u tools/fp4_half_ab.py "6 7 8 9" 3 2 > gpurun_out/r06_c_fp4_half.log 2>&1 || { echo FP4AB FAIL; tail -20 gpurun_out/r06_c_fp4_half.log; exit 1; }
cat gpurun_out/r06_c_fp4_half.log
