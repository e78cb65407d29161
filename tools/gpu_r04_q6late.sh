# Round 4: q6 digit records stored one phase late (after the next sub-tile's dz phase), so they
# drain while it is quantised -- tests on the tree, then kernel stats O (HEAD) vs C (the tree).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_q6_handoff.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_q6late_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_q6late_tests.log; [ $rc = 0 ] || exit 1
AB_GREP="q6_k" LIBS="O=ab/O/libbnn.so C=ab/C/libbnn.so" bash tools/gpu_r04_ab.sh
