# Round-3: statistics epilogues as their own kernel instances (the plain FP6 / int8 kernels as
# before the statistics work): pixel / hand-off / FP6 tests, A (BNN_PIX_STATS=0) / B wide stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_pixels.py tests/test_gpu_q6_handoff.py tests/test_gpu_fp6.py > gpurun_out/sp_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/sp_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
BNN_PIX_STATS=0 AB_TOP=8 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=8 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
