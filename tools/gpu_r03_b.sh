# Round-3 GPU call B: the reworked whole-net / wide-trace parity tests, then A/B kernel stats of
# the wide step (A = the round-2 q6 kernels, B = this tree).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_net_configs.py tests/test_gpu_wide_trace.py > gpurun_out/r03_b_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "PASSED|FAILED|Net r=3|  drop-in|  fused|^E  " gpurun_out/r03_b_tests.log | cut -c1-600 | head -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab_stats.sh A=ab/A/libbnn.so B=distributed-mnist-bnns_amd/lib/libbnn.so
