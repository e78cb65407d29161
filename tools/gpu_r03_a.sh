# Round-3 GPU call A: every -m gpu test (verbose, prints kept), then SQ PMC passes over the wide
# step's BatchNorm kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR|passed|failed|wide trace|Net r=3|M=[0-9]|  \{" gpurun_out/r03_gpu_tests.log | tail -80
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_pmc_bench.sh wide bn_ > gpurun_out/pmc_wide_bn.txt 2>&1 || { echo PMC FAIL; tail -20 gpurun_out/pmc_wide_bn.txt; exit 1; }
cat gpurun_out/pmc_wide_bn.txt | head -120
exit $rc
