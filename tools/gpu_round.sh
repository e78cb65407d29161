# GPU session: parity tests, GEMM sweep, bench (with kernel timing), rocprof stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1; echo "PARITY EXIT $?"; tail -3 gpurun_out/parity.log
grep -E "FAIL|Error" gpurun_out/parity.log | head -20
timeout -k 10 300 python -u tools/gemm_sweep.py --reps 3 > gpurun_out/sweep.log 2>&1 || { echo SWEEP FAIL; tail -20 gpurun_out/sweep.log; exit 1; }
cat gpurun_out/sweep.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
