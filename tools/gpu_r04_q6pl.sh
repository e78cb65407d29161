# Round 4: q6_block_pre with planes 0-2 from P in a rolled loop and plane 3 from a pre-biased Q (no
# per-pair select) -- the q6 / head / wide-step tests on the tree, then kernel stats O (HEAD
# before it) vs B (the tree).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_q6_handoff.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_q6pl_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_q6pl_tests.log; [ $rc = 0 ] || exit 1
AB_GREP="q6_k" LIBS="O=ab/O/libbnn.so B=ab/B/libbnn.so" bash tools/gpu_r04_ab.sh
