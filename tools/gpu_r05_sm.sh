# The same-mask loss test of the bench workload (with its permuted-batch calibration), then the N > 1
# bench path rehearsed with 2 gloo ranks on the box's one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu "tests/test_gpu_wide_step.py::test_wide_bench_loss_same_masks" > gpurun_out/r05_same_masks.log 2>&1; rc=$?
grep -E "libbnn|torch fp32|permuted|relative gap|tail means|passed|failed" gpurun_out/r05_same_masks.log | cut -c1-400
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_rehearse_n2.sh
