# Round-3: FP4 panel staging for the FP6 GEMM: FP6 tests, the wide bench line, MLP line, kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp6.py tests/test_gpu_fused.py > gpurun_out/pan_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/pan_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/pan_wide.log 2>&1 || { tail -5 gpurun_out/pan_wide.log; exit 1; }
tail -1 gpurun_out/pan_wide.log | cut -c1-200
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/pan_mlp.log 2>&1 || exit 1
tail -1 gpurun_out/pan_mlp.log | cut -c1-200
AB_TOP=14 bash tools/gpu_ab_stats.sh wide_pan=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=14 BENCH_ARGS="--config mlp" bash tools/gpu_ab_stats.sh mlp_pan=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
