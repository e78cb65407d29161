# config 2's two-rank exchange with the hook / write / launch order recorded
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ddp_config2_diag.py 3 > gpurun_out/r05_y_c2.log 2>&1; rc=$?
echo "exit $rc"; grep -v amdgpu gpurun_out/r05_y_c2.log | grep -v "^\[" | grep -v "hand-offs" | cut -c1-1500
