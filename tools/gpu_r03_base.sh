# Round-3 baseline on a fresh box: every -m gpu test, the default bench line, the MLP (config 3)
# and BinCNN (config 4) lines, and kernel-trace stats of the three steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/base_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED" gpurun_out/base_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/base_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/base_bench.log; exit 1; }
tail -1 gpurun_out/base_bench.log | cut -c1-400
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/base_mlp.log 2>&1 || exit 1
tail -1 gpurun_out/base_mlp.log | cut -c1-300
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/base_cnn.log 2>&1 || exit 1
tail -1 gpurun_out/base_cnn.log | cut -c1-300
AB_TOP=12 bash tools/gpu_ab_stats.sh wide=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=14 BENCH_ARGS="--config mlp" bash tools/gpu_ab_stats.sh mlp=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=14 BENCH_ARGS="--config cnn" bash tools/gpu_ab_stats.sh cnn=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
