# Round 4: the head's q6 pass with dY4 rows prefetched a sub-tile ahead (tree = A) -- its tests,
# then kernel stats of O (HEAD before it), A, and timing-only builds nq (no quantisation) and ns
# (no digit stores).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_q6_handoff.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_q6d4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_q6d4_tests.log; [ $rc = 0 ] || exit 1
AB_GREP="q6_k" LIBS="O=ab/O/libbnn.so A=ab/A/libbnn.so nq=ab/nq/libbnn.so ns=ab/ns/libbnn.so" bash tools/gpu_r04_ab.sh
