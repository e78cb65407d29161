# BinCNN artifacts: conv parity tests, eager and HIP-graph bench lines, rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or cnn" > gpurun_out/cnn_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/cnn_tests.log; exit 1; }
tail -1 gpurun_out/cnn_tests.log
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 > gpurun_out/cnn_eager.log 2>&1 || { echo EAGER FAIL; tail -5 gpurun_out/cnn_eager.log; exit 1; }
grep "^{" gpurun_out/cnn_eager.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --graph --no-cpu-baseline --no-gpu-torch > gpurun_out/cnn_graph.log 2>&1 || { echo GRAPH FAIL; tail -5 gpurun_out/cnn_graph.log; exit 1; }
grep "^{" gpurun_out/cnn_graph.log | cut -c1-200
rm -rf gpurun_out/prof_cnn
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn -o run --output-format csv -- python bench.py --config cnn --steps 20 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > gpurun_out/cnn_prof.log 2>&1 || { echo PROF FAIL; tail -5 gpurun_out/cnn_prof.log; exit 1; }
echo done
