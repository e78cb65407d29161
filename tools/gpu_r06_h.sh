# Round 6, call H: agent-scope atomic loads on every compact conv reader by default (BN2_LOADS=2);
# GraphedStep replays the fp32-image recognition it saw in its warm-up (guarded); DDP around the
# drop-in modules.  The determinism-sensitive tests in one run, then the one-rank RCCL probe.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_graph.py tests/test_gpu_rccl.py tests/test_gpu_parallel.py tests/test_gpu_ddp_dropin.py \
  tests/test_gpu_pixels.py > gpurun_out/r06_h_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "PASS|FAIL|Error|assert" gpurun_out/r06_h_gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r06_h_gpu_tests.log | tail -3
timeout -k 10 300 python -u tools/det_rccl_probe.py 3 > gpurun_out/r06_h_det_rccl.log 2>&1 || { echo DET FAIL; tail -20 gpurun_out/r06_h_det_rccl.log; exit 1; }
grep -E "^(eager|exchange|graph)" gpurun_out/r06_h_det_rccl.log
