# Round 4 GPU call: conv1's filter gradient fused with its BatchNorm2d backward (c1bn hand-off) --
# tests (hand-off vs unfused, the BinCNN parity suite), BinCNN kernel stats, bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cnn_parity.py tests/test_gpu_fused.py tests/test_gpu_graph.py -k "bn2d or batchnorm2d or cnn or CNN or conv" -q --timeout 300 --timeout-method thread > gpurun_out/r04_c1bn_tests.log 2>&1
rc=$?; echo "C1BN TESTS EXIT $rc"; tail -3 gpurun_out/r04_c1bn_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_stats.sh cnnc1bn --config cnn > gpurun_out/cnnc1bn.txt 2>&1 || { echo "CNN STATS FAIL"; tail -5 gpurun_out/cnnc1bn.txt; exit 1; }
head -18 gpurun_out/cnnc1bn.txt | cut -c1-140
timeout -k 10 300 python bench.py --config cnn --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench3.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench3.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --graph --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench3_graph.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench3_graph.log | cut -c1-200
