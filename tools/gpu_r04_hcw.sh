# Round 4: the head's statistics pass (bn_head_reduce_k) at 2 columns per thread (-DHR_CW=2: 142
# VGPRs, 3 waves per SIMD; c2o4 also forced to 4 waves) -- the head tests on c2, then kernel stats
# of the bench step, O (HEAD: 4 columns per thread, 214 VGPRs, 2 waves) vs c2 vs c2o4. (The variant was a patch over HEAD, reverted after this run; its source is not in the tree.)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BNN_LIB=$R/ab/c2/libbnn.so timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_hcw_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_hcw_tests.log; [ $rc = 0 ] || exit 1
AB_GREP="bn_head_reduce" LIBS="O=ab/O/libbnn.so c2=ab/c2/libbnn.so c2o4=ab/c2o4/libbnn.so" bash tools/gpu_r04_ab.sh
