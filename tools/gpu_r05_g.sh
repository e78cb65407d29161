# Round 5: the DDP / GradExchange test against the exact rank average, then the full GPU suite + smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py -v --timeout 300 --timeout-method thread > gpurun_out/r05_g_par.log 2>&1
echo "PAR exit $?"; grep -E "PASS|FAIL|Error" gpurun_out/r05_g_par.log | cut -c1-500 | tail -12
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --deselect tests/test_gpu_parallel.py > gpurun_out/r05_g_suite.log 2>&1
rc=$?; echo "SUITE exit $rc"; tail -6 gpurun_out/r05_g_suite.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
