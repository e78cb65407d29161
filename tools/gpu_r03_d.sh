# Round-3 GPU call D: the quantising-BN-backward tests (staged whole-line digit stores), then A/B/C
# kernel stats (A = r02, B = tree with the head at 3 waves/SIMD, C = head at 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gpu_q6_handoff.py tests/test_gpu_head.py tests/test_gpu_z16.py tests/test_gpu_fused.py \
  tests/test_gpu_fp6.py tests/test_gpu_wide_trace.py tests/test_gpu_training.py tests/test_gpu_loss_curve.py -s > gpurun_out/r03_d_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  |window mean|first exact" gpurun_out/r03_d_tests.log | cut -c1-300 | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_TOP=8 bash tools/gpu_ab_stats.sh A=ab/A/libbnn.so B=distributed-mnist-bnns_amd/lib/libbnn.so C=ab/C/libbnn.so
