# Round-3: q6 BN backward without LDS atomics (+ hi staging swizzle), by-row pooled BatchNorm2d
# passes: every -m gpu test, then A (HEAD library) / B (tree) kernel stats of the wide and CNN steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/q6b_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/q6b_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
AB_TOP=8 bash tools/gpu_ab_stats.sh A=ab/A/libbnn.so B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=14 BENCH_ARGS="--config cnn" bash tools/gpu_ab_stats.sh cA=ab/A/libbnn.so cB=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
