# Round-3: compact conv outputs (CNN) + graph-mode MLP/CNN benches + kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/cq_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/cq_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/cq_cnn.log 2>&1 || { tail -5 gpurun_out/cq_cnn.log; exit 1; }
tail -1 gpurun_out/cq_cnn.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --graph --steps 100 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/cq_cnn_g.log 2>&1 || { tail -5 gpurun_out/cq_cnn_g.log; exit 1; }
tail -1 gpurun_out/cq_cnn_g.log | cut -c1-200
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/cq_mlp_g.log 2>&1 || { tail -5 gpurun_out/cq_mlp_g.log; exit 1; }
tail -1 gpurun_out/cq_mlp_g.log | cut -c1-200
AB_TOP=20 BENCH_ARGS="--config cnn" bash tools/gpu_ab_stats.sh cnn_q=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=30 BENCH_ARGS="--config mlp --graph" bash tools/gpu_ab_stats.sh mlp_graph=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
