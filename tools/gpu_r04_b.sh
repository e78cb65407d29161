# Round 4 GPU call: q6 shuffle-maxima variant tests + A/B, and the pixel-GEMM diagnostic timings.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for lib in distributed-mnist-bnns_amd/lib/libbnn.so ab/nomain/libbnn.so ab/nostore/libbnn.so distributed-mnist-bnns_amd/lib/libbnn.so; do
  BNN_LIB=$R/$lib timeout -k 10 120 python tools/pix_diag.py >> gpurun_out/r04_pix_diag.log 2>&1 || { echo PIXDIAG FAIL; tail -5 gpurun_out/r04_pix_diag.log; exit 1; }
done
cat gpurun_out/r04_pix_diag.log | grep "per launch"
BNN_LIB=$R/ab/shfl/libbnn.so timeout -k 10 500 python -u -m pytest tests/test_gpu_q6_handoff.py tests/test_gpu_fused.py tests/test_gpu_head.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r04_shfl_tests.log 2>&1; echo "SHFL TESTS $?"; tail -2 gpurun_out/r04_shfl_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_wide_trace.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r04_tree_tests.log 2>&1; echo "TREE TESTS $?"; tail -2 gpurun_out/r04_tree_tests.log
AB_GREP="q6_k<0" LIBS="A=distributed-mnist-bnns_amd/lib/libbnn.so B=ab/shfl/libbnn.so" bash tools/gpu_r04_ab.sh
