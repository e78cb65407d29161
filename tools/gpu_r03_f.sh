# Round-3 GPU call F: the whole -m gpu suite on the atomic-max / staged-store q6 kernels, then A/B stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_f_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/r03_f_tests.log | cut -c1-300 | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_TOP=8 bash tools/gpu_ab_stats.sh A=ab/A/libbnn.so B=distributed-mnist-bnns_amd/lib/libbnn.so
