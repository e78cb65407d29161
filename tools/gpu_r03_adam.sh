# Round-3: Adam + clamp + FP4 re-pack on 256 x 256 tiles: its tests, A (64 x 64 tiles) / B wide stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_graph.py > gpurun_out/ad_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/ad_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
BNN_ADAM_TILE256=0 AB_TOP=10 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
BNN_ADAM_TILE256=1 AB_TOP=10 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
