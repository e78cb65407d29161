# Round-3: bn1's forward statistics from the pixel GEMM's epilogue: pixel tests, A (BNN_PIX_STATS=0)
# / B wide kernel stats, the full -m gpu suite, then the wide bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_pixels.py > gpurun_out/ps_pix.log 2>&1
rc=$?; echo "PIXEL TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/ps_pix.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
BNN_PIX_STATS=0 AB_TOP=14 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=14 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/ps_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/ps_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/ps_wide.log 2>&1 || { tail -5 gpurun_out/ps_wide.log; exit 1; }
tail -1 gpurun_out/ps_wide.log | cut -c1-200
