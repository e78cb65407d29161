# Round 4: the whole-step parity tests at the benched sizes (config 5 B=65536 vs float64, the
# bench's loss beside the reference semantics, the BinCNN trace and B=4096 step, the dropout-on
# loss curve), then a baseline bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_wide_step.py tests/test_gpu_cnn_parity.py tests/test_gpu_loss_curve.py "tests/test_gpu_parity.py::test_compact_conv_falls_back_when_refused" "tests/test_gpu_graph.py::test_device_step_eager_with_missing_gradients" -v -s --timeout 300 --timeout-method thread > gpurun_out/r04_parity.log 2>&1
rc=$?; echo "PARITY EXIT $rc"; grep -E "PASS|FAIL|Error|config 5|BinCNN|mean of|window|libbnn|torch" gpurun_out/r04_parity.log | cut -c1-400 | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-gpu-torch > gpurun_out/r04_base_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r04_base_bench.log; exit 1; }
tail -1 gpurun_out/r04_base_bench.log | cut -c1-400
