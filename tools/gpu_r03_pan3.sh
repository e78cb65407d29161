# Round-3: every FP6 B operand in the panel layout (weights' transposes from the fused Adam re-pack,
# small-batch BN apply-packs): every -m gpu test; wide / MLP-graph / CNN benches + stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/p3_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/p3_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/p3_wide.log 2>&1 || { tail -5 gpurun_out/p3_wide.log; exit 1; }
tail -1 gpurun_out/p3_wide.log | cut -c1-200
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/p3_mlp_g.log 2>&1 || { tail -5 gpurun_out/p3_mlp_g.log; exit 1; }
tail -1 gpurun_out/p3_mlp_g.log | cut -c1-200
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/p3_mlp.log 2>&1 || { tail -5 gpurun_out/p3_mlp.log; exit 1; }
tail -1 gpurun_out/p3_mlp.log | cut -c1-200
AB_TOP=16 BENCH_ARGS="--config mlp --graph" bash tools/gpu_ab_stats.sh mlp_p3=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=10 bash tools/gpu_ab_stats.sh wide_p3=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
