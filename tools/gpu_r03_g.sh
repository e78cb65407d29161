# Round-3 GPU call G: the RCCL test and the exchange trace with the high-priority RCCL stream.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/r03_g_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; tail -2 gpurun_out/r03_g_tests.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_exchange
bash tools/gpu_r03_e.sh
grep -c . gpurun_out/comm_overlap.txt
