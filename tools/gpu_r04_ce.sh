# Round 4: the training loop's criterion on libbnn (bnn_cross_entropy_*) -- its tests and the graph
# tests, then the bench lines it changes (wide, BinCNN eager / graph, MLP eager / graph).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_ce_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r04_ce_tests.log; [ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/r04_ce_tests.log | head; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/r04_ce_wide.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/r04_ce_cnn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --graph --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/r04_ce_cnn_g.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/r04_ce_mlp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/r04_ce_mlp_g.log 2>&1 || exit 1
for f in wide cnn cnn_g mlp mlp_g; do echo "$f: $(tail -1 gpurun_out/r04_ce_$f.log | grep -o '"ms_per_step": [0-9.]*')"; done
bash tools/gpu_stats.sh ce_cnn --config cnn --graph > gpurun_out/r04_ce_cnn_stats.txt 2>&1 || exit 1
grep -E "cross_entropy|ce_|nll|softmax|Fill|kernel time" gpurun_out/r04_ce_cnn_stats.txt | cut -c1-150
