# Round-3: the full -m gpu suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/t_all.log 2>&1
rc=$?; echo "ALL TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/t_all.log | cut -c1-300 | head -20
exit $rc
