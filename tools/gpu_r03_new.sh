# GPU session: the round-3 parity tests (wide trace, Net configs, RCCL one-rank, config-5 dW, graph quirk).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_wide_trace.py tests/test_gpu_net_configs.py tests/test_gpu_rccl.py \
  "tests/test_gpu_fused.py::test_wide_backward_heavy_tailed_vs_float64" \
  "tests/test_gpu_parity.py::test_linear_matches_reference_golden" tests/test_gpu_graph.py \
  ${PYTEST_ARGS} > gpurun_out/r03_new_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "PASSED|FAILED|ERROR|wide trace|Net r=3|M=|step" gpurun_out/r03_new_tests.log | tail -60
exit $rc
