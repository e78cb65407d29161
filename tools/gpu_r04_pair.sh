# Round 4: 2-byte GEMM outputs (int16 z16, s20) stored two 32-column patches at a time (whole
# 128-B lines, 16-B stores) -- the z16 / s20 / pixel / parity tests on the tree, the fc3 FP4 GEMM
# alone (O = HEAD before it, D = the tree), then kernel stats of the wide step O vs D.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_z16.py tests/test_gpu_s20.py tests/test_gpu_pixels.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_pair_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_pair_tests.log; [ $rc = 0 ] || exit 1
for lib in ab/O/libbnn.so ab/D/libbnn.so ab/O/libbnn.so ab/D/libbnn.so; do
  BNN_LIB=$R/$lib timeout -k 10 120 python tools/fp4_diag.py >> gpurun_out/r04_pair_fp4.log 2>&1 || { echo FP4DIAG FAIL; tail -5 gpurun_out/r04_pair_fp4.log; exit 1; }
done
grep "per launch" gpurun_out/r04_pair_fp4.log
AB_GREP="gemm_fp4|gemm_i8_v2_k<1, 1" LIBS="O=ab/O/libbnn.so D=ab/D/libbnn.so" bash tools/gpu_r04_ab.sh
