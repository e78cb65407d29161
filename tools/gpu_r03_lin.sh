# Round-3: narrow fp32 Linear for the BinCNN classifier: its tests + the CNN parity tests, then the
# CNN bench line and kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_linear_small.py tests/test_gpu_parity.py > gpurun_out/lin_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/lin_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/lin_cnn.log 2>&1 || { tail -5 gpurun_out/lin_cnn.log; exit 1; }
tail -1 gpurun_out/lin_cnn.log | cut -c1-200
AB_TOP=16 BENCH_ARGS="--config cnn --steps 7 --warmup 3" bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
