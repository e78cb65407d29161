# Round 6, call B: workgroup placement probe, the FP6 half-tile A/B, torch BatchNorm1d layouts,
# the DDP drop-in test (z1-anchored) and the dropout loss-curve test (8 seeds, s.e. bar).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 60 tools/probes/probe_wg_placement > gpurun_out/r06_b_wg_placement.log 2>&1 || { echo PROBE FAIL; tail gpurun_out/r06_b_wg_placement.log; exit 1; }
cat gpurun_out/r06_b_wg_placement.log
timeout -k 10 300 python -u tools/fp6_half_ab.py "0:0 1:0 1:40 1:80 1:130 1:200" 3 2 > gpurun_out/r06_b_fp6_half.log 2>&1 || { echo HALF FAIL; tail -20 gpurun_out/r06_b_fp6_half.log; exit 1; }
cat gpurun_out/r06_b_fp6_half.log
timeout -k 10 200 python -u tools/torch_bn_layout_probe.py > gpurun_out/r06_b_torch_bn_layout.log 2>&1 || { echo BNPROBE FAIL; tail -20 gpurun_out/r06_b_torch_bn_layout.log; exit 1; }
cat gpurun_out/r06_b_torch_bn_layout.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp_dropin.py "tests/test_gpu_loss_curve.py::test_mnist_loss_curve_dropout" -m gpu -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/r06_b_tests.log 2>&1; rc=$?
echo "TESTS exit $rc"; grep -E "passed|failed|\[org\]|\[frozen\]|accuracy" gpurun_out/r06_b_tests.log | tail -12; grep -E "^E " gpurun_out/r06_b_tests.log | cut -c1-300 | head -12
