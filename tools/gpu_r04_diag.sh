# Round 4: the config-5 whole-step test (Hardtanh-boundary columns reported, torch fp32 for scale)
# and the BinCNN parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -v -s --timeout 280 --timeout-method thread > gpurun_out/r04_diag_a.log 2>&1
echo "A exit $?"; grep -E "config 5|libbnn vs|Hardtanh-boundary|torch fp32 vs|per-row|update max|Error" gpurun_out/r04_diag_a.log | cut -c1-1200
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn_parity.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r04_diag_c.log 2>&1
echo "C exit $?"; grep -E "PASS|FAIL|BinCNN|libbnn vs|torch fp32 vs|update max|Error" gpurun_out/r04_diag_c.log | cut -c1-900
