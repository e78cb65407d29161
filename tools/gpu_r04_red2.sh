# Round 4 GPU call: the BatchNorm-reduction occupancy A/B of the wide step (variants rebuilt from the
# tree), then plain BinCNN bench lines (eager and graph).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/gpu_r04_red.sh || exit 1
timeout -k 10 300 python bench.py --config cnn --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --config cnn --graph --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench_graph.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench_graph.log | cut -c1-300
