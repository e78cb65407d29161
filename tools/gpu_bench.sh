set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1; echo "PARITY EXIT $?"; tail -2 gpurun_out/parity.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
