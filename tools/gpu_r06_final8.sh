# Round-6 last check on HEAD (on HEAD with QC_RT_SMALL = 2): GPU suite A + B, smoke,
# the default bench line and the config-3 graph line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_final8_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_final8_gpu_tests_a.log | tail -1; grep -E "^FAILED" gpurun_out/r06_final8_gpu_tests_a.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -q -rf --timeout 600 --timeout-method thread > gpurun_out/r06_final8_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r06_final8_gpu_tests_b.log | tail -1; grep -E "^FAILED" gpurun_out/r06_final8_gpu_tests_b.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06_final8_smoke.log 2>&1 || { echo SMOKE FAIL; tail -5 gpurun_out/r06_final8_smoke.log; exit 1; }
tail -1 gpurun_out/r06_final8_smoke.log
timeout -k 10 300 python bench.py --config mlp --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_final8_bench_mlpgraph.log 2>&1 || exit 1
echo "mlp --graph: $(tail -1 gpurun_out/r06_final8_bench_mlpgraph.log | grep -o '"ms_per_step": [0-9.]*')"
timeout -k 10 500 python bench.py > gpurun_out/r06_final8_bench_wide.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r06_final8_bench_wide.log; exit 1; }
tail -1 gpurun_out/r06_final8_bench_wide.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_final8_bench_cnngraph.log 2>&1 || exit 1
echo "cnn --graph: $(tail -1 gpurun_out/r06_final8_bench_cnngraph.log | grep -o '"ms_per_step": [0-9.]*')"
