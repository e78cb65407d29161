# Round 4: the GEMM epilogue filling every patch of a tile row before storing, s20 stored as patch
# pairs (D = tree) against O (HEAD before it): the z16 / s20 / pixel / parity tests, the fc3 FP4
# GEMM alone, kernel stats of the wide step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_z16.py tests/test_gpu_s20.py tests/test_gpu_pixels.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_pair2_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r04_pair2_tests.log; [ $rc = 0 ] || exit 1
for lib in ab/O/libbnn.so ab/D/libbnn.so ab/O/libbnn.so ab/D/libbnn.so; do
  BNN_LIB=$R/$lib timeout -k 10 120 python tools/fp4_diag.py >> gpurun_out/r04_pair2_fp4.log 2>&1 || { echo FP4DIAG FAIL; tail -5 gpurun_out/r04_pair2_fp4.log; exit 1; }
done
grep "per launch" gpurun_out/r04_pair2_fp4.log
AB_GREP="gemm_fp4|gemm_i8_v2_k<1, 1" LIBS="O=ab/O/libbnn.so D=ab/D/libbnn.so" bash tools/gpu_r04_ab.sh
