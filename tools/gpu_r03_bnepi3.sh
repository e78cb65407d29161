# Round-3: FP6 dX epilogue statistics taken from the accumulators before any C store: hand-off tests,
# A (BNN_BN_EPI=0) / B (BNN_BN_EPI=1) wide kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_q6_handoff.py tests/test_gpu_pixels.py > gpurun_out/be3_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/be3_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
BNN_BN_EPI=0 AB_TOP=12 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
BNN_BN_EPI=1 AB_TOP=12 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
