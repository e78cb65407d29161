set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python tools/ddp_cnn_diag.py > gpurun_out/r05_h_ddpcnn.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r05_h_ddpcnn.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py -v --timeout 300 --timeout-method thread > gpurun_out/r05_h_par.log 2>&1
echo "PAR exit $?"; grep -E "PASS|FAIL|AssertionError: \(" gpurun_out/r05_h_par.log | cut -c1-300 | tail -12
