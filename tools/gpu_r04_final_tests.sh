# Round-4 final artifacts, part 1: every -m gpu test and smoke() on HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04_final_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -2 gpurun_out/r04_final_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r04_final_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r04_final_smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r04_final_smoke.log; exit 1; }
tail -1 gpurun_out/r04_final_smoke.log
