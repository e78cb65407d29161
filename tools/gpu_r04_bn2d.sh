# Round 4 GPU call: row forms of the pooled BatchNorm2d passes -- tests, BinCNN kernel stats, bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cnn_parity.py tests/test_gpu_fused.py -k "bn2d or batchnorm2d or cnn or CNN or conv" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_bn2d_tests.log 2>&1
rc=$?; echo "BN2D TESTS EXIT $rc"; tail -3 gpurun_out/r04_bn2d_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_stats.sh cnnrows --config cnn > gpurun_out/cnnrows.txt 2>&1 || { echo "CNN STATS FAIL"; tail -5 gpurun_out/cnnrows.txt; exit 1; }
head -16 gpurun_out/cnnrows.txt | cut -c1-140
timeout -k 10 300 python bench.py --config cnn --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench2.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench2.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --graph --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench2_graph.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench2_graph.log | cut -c1-200
