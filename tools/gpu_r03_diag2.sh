set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/fp6_diag.py 65536 8192 8192 3 10 7 5 97 98 95 91 > gpurun_out/fp6_diag2.log 2>&1; rc=$?
cat gpurun_out/fp6_diag2.log; exit $rc
