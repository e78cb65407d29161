# Round 4: the head q6 pass with its dY4 rows staged a sub-tile ahead by LDS-DMA -- head / q6 / fused
# / wide tests on the tree (E), then kernel stats O (HEAD before it) vs E.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_q6_handoff.py tests/test_gpu_fused.py tests/test_gpu_wide_step.py tests/test_gpu_net_configs.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_d4dma_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r04_d4dma_tests.log; [ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/r04_d4dma_tests.log | head; exit 1; }
AB_GREP="q6_k" LIBS="O=ab/O/libbnn.so E=ab/E/libbnn.so" bash tools/gpu_r04_ab.sh
