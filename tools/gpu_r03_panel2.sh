# Round-3: panel transpose from the fused BN apply-pack; every -m gpu test; wide bench + stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/pan2_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/pan2_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/pan2_wide.log 2>&1 || { tail -5 gpurun_out/pan2_wide.log; exit 1; }
tail -1 gpurun_out/pan2_wide.log | cut -c1-200
AB_TOP=14 bash tools/gpu_ab_stats.sh wide_pan2=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 300 python3 tools/fp6_diag.py 65536 8192 8192 3 10 7 5 14 15 98 95 > gpurun_out/fp6_diag2.log 2>&1; rc=$?
cat gpurun_out/fp6_diag2.log; exit $rc
