# the whole GPU suite on HEAD in two parts (-v: one line per test; the long whole-step tests with -s
# so they print as they go), then smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r05_full4_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r05_full4_gpu_tests_a.log | tail -3; grep -E "^FAILED|Error" gpurun_out/r05_full4_gpu_tests_a.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r05_full4_smoke.log 2>&1; echo "SMOKE exit $?"; tail -2 gpurun_out/r05_full4_smoke.log
