# Round-3: config 3 (MLP r=3, B=4096) and config 4 (BinCNN) as HIP-graph replays + kernel stats;
# PMC passes over the quantising BatchNorm backward of the wide step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/g_mlp.log 2>&1 || { tail -5 gpurun_out/g_mlp.log; exit 1; }
tail -1 gpurun_out/g_mlp.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --graph --steps 100 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/g_cnn.log 2>&1 || { tail -5 gpurun_out/g_cnn.log; exit 1; }
tail -1 gpurun_out/g_cnn.log | cut -c1-200
AB_TOP=30 BENCH_ARGS="--config mlp --graph" bash tools/gpu_ab_stats.sh mlp_graph=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
bash tools/gpu_pmc_bench.sh q6 bn_bwd_apply_q6 || exit 1
