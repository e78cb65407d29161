# Round-3 GPU call C: the teacher-forced / free-running wide-trace tests, then A/B/diag kernel stats
# of the wide step's quantising BatchNorm backward (A = r02, B = tree, D1 = no digit stores,
# D2 = no quantisation).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_wide_trace.py > gpurun_out/r03_c_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "PASSED|FAILED|free-running|^E  " gpurun_out/r03_c_tests.log | cut -c1-400 | head -30
grep -E "  drop-in|  fused" gpurun_out/r03_c_tests.log | sed -E "s/'g:[a-z0-9.]+': [0-9.e-]+, //g" | cut -c1-330 | head -24
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_TOP=6 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so D1=ab/D1/libbnn.so D2=ab/D2/libbnn.so
