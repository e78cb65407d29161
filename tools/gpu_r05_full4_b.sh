# the long whole-step GPU tests (-s: they print per step / per check)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
timeout -k 10 60 python -u -m pytest "tests/test_gpu_parity.py::test_empty_and_single_sample_batches" -q --timeout 50 --timeout-method thread > gpurun_out/r05_full4_fix.log 2>&1; echo "FIX exit $?"; tail -1 gpurun_out/r05_full4_fix.log
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/r05_full4_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r05_full4_gpu_tests_b.log | tail -3; grep -E "^FAILED|Error" gpurun_out/r05_full4_gpu_tests_b.log | cut -c1-250 | head -12
