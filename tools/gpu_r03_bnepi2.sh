# Round-3: batched x loads in the FP6 statistics epilogue: the epilogue / hand-off GPU tests, then
# A (BNN_BN_EPI=0) / B wide kernel stats and the bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_q6_handoff.py tests/test_gpu_pixels.py tests/test_gpu_z16.py > gpurun_out/be2_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/be2_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
BNN_BN_EPI=0 AB_TOP=12 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=12 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/be2_wide.log 2>&1 || { tail -5 gpurun_out/be2_wide.log; exit 1; }
tail -1 gpurun_out/be2_wide.log | cut -c1-200
