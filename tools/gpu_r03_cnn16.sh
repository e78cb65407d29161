# Round-3: BinCNN with int16 conv outputs for both layers (+ the stats-reduce index fix): CNN tests,
# A (HEAD library) / B (tree) CNN kernel stats, the CNN bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_q6_handoff.py tests/test_gpu_head.py > gpurun_out/c16_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/c16_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
AB_TOP=14 BENCH_ARGS="--config cnn" bash tools/gpu_ab_stats.sh cA=ab/A/libbnn.so cB=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/c16_cnn.log 2>&1 || exit 1
tail -1 gpurun_out/c16_cnn.log | cut -c1-200
