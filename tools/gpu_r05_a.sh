# Round 5: the config-5 whole-step test anchored on libbnn's Hardtanh decisions, with the
# backward-GEMM calibration runs (fp32 / FP6 emulations), and the BinCNN parity tests (fp32-GEMM
# calibration of the conv backward, conv biases held to the reference's trajectory).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -v -s --timeout 380 --timeout-method thread > gpurun_out/r05_a_wide.log 2>&1
echo "A exit $?"; grep -E "config 5|Hardtanh|per-row|gradient|weight|bias|update max|Error|assert" gpurun_out/r05_a_wide.log | cut -c1-400 | head -60
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn_parity.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r05_a_cnn.log 2>&1
echo "C exit $?"; grep -E "PASS|FAIL|BinCNN|libbnn vs|fp32-GEMM|update max|Error|assert" gpurun_out/r05_a_cnn.log | cut -c1-900 | head -40
