# Round 4 GPU call: placeholders without fill kernels, bias carried without snapshot copies --
# the compact-form and CNN tests, then wide and BinCNN bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_s20.py tests/test_gpu_z16.py tests/test_gpu_parity.py tests/test_gpu_cnn_parity.py tests/test_gpu_graph.py tests/test_gpu_q6_handoff.py tests/test_gpu_head.py -q --timeout 300 --timeout-method thread > gpurun_out/r04_misc_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/r04_misc_tests.log; grep -E "^FAILED" gpurun_out/r04_misc_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cnn --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench4.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench4.log | cut -c1-200
timeout -k 10 300 python bench.py --config cnn --graph --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_cnn_bench4_graph.log 2>&1 && tail -1 gpurun_out/r04_cnn_bench4_graph.log | cut -c1-200
timeout -k 10 400 python bench.py --no-gpu-torch --no-cpu-baseline > gpurun_out/r04_wide_bench4.log 2>&1 && tail -1 gpurun_out/r04_wide_bench4.log | cut -c1-200
