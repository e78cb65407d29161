set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1; rc=$?; echo "PARITY EXIT $rc"; tail -3 gpurun_out/parity.log
[ $rc -eq 0 ] || grep -E "Error|assert|FAIL" gpurun_out/parity.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --config cnn --steps 10 --warmup 2 > gpurun_out/bench_cnn.log 2>&1 && tail -1 gpurun_out/bench_cnn.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_wide.log 2>&1 && tail -1 gpurun_out/bench_wide.log
