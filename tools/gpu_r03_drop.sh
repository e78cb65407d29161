# Round-3: bn3's forward statistics (of drop(z3)) from fc3's FP4 epilogue: z16 / training / graph
# tests, A (BNN_FP4_STATS=0) / B wide kernel stats, the full -m gpu suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_z16.py tests/test_gpu_training.py tests/test_gpu_graph.py tests/test_gpu_q6_handoff.py > gpurun_out/dr_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/dr_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
BNN_FP4_STATS=0 AB_TOP=14 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=14 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/dr_all.log 2>&1
rc=$?; echo "ALL TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/dr_all.log | cut -c1-300 | head -20
exit $rc
