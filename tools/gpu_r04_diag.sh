# Round 4: the config-5 whole-step test with its fp32 calibration, with bn1's forward statistics from
# fc1's epilogue (default) and from a pass over the stored z1 (BNN_PIX_STATS=0); the BinCNN tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -v -s --timeout 280 --timeout-method thread > gpurun_out/r04_diag_a.log 2>&1
echo "A exit $?"; grep -E "config 5|libbnn vs|torch fp32 vs|per-row|update max|Error" gpurun_out/r04_diag_a.log | cut -c1-900
BNN_PIX_STATS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -v -s --timeout 280 --timeout-method thread > gpurun_out/r04_diag_b.log 2>&1
echo "B exit $?"; grep -E "config 5|libbnn vs|torch fp32 vs|per-row|update max|Error" gpurun_out/r04_diag_b.log | cut -c1-900
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn_parity.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r04_diag_c.log 2>&1
echo "C exit $?"; grep -E "PASS|FAIL|BinCNN|libbnn vs|torch fp32 vs|update max|Error" gpurun_out/r04_diag_c.log | cut -c1-900
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -v --timeout 200 --timeout-method thread > gpurun_out/r04_diag_d.log 2>&1
echo "D exit $?"; grep -E "PASS|FAIL|Error" gpurun_out/r04_diag_d.log | cut -c1-300 | tail -12
BNN_DROP_BITS=0 bash tools/gpu_stats.sh r04_nobits > gpurun_out/r04_stats_nobits.txt 2>&1 && head -22 gpurun_out/r04_stats_nobits.txt && grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_r04_nobits.log
bash tools/gpu_stats.sh r04_bits > gpurun_out/r04_stats_bits.txt 2>&1 && head -22 gpurun_out/r04_stats_bits.txt && grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_r04_bits.log
