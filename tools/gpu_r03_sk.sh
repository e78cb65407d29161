# Round-3: FP6 split-K plan + BN final merges: the whole -m gpu suite, MLP bench + kernel stats,
# interleaved FP6 variant timing on the wide dX shape (2- vs 3-stage rings).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/sk_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/sk_mlp.log 2>&1 || exit 1
tail -1 gpurun_out/sk_mlp.log | cut -c1-200
AB_TOP=24 BENCH_ARGS="--config mlp" bash tools/gpu_ab_stats.sh mlp_sk=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 300 python3 tools/fp6_diag.py 65536 8192 8192 3 10 7 5 10 97 98 95 > gpurun_out/fp6_var.log 2>&1; rc=$?
cat gpurun_out/fp6_var.log; exit $rc
