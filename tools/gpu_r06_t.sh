# Round 6, call T: DDP around the drop-in modules with bnn_amd.nn.BatchNorm1d (org-bn), the graph
# tests after the per-capture guard reset, the drop-in BatchNorm tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ddp_dropin.py \
  tests/test_gpu_graph.py tests/test_gpu_bn_dropin.py > gpurun_out/r06_t_gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r06_t_gpu_tests.log | tail -1; grep -E "^\[org|FAILED|^E  " gpurun_out/r06_t_gpu_tests.log | cut -c1-220 | head -30
exit $rc
