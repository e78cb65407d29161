# within-step re-reads of the compact conv output by the BatchNorm2d forward under contention
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
RACE_MITIGATE="reread" timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_p_reread.log 2>&1; rc=$?
echo "== reread exit $rc: $(grep -c 'first difference' gpurun_out/r05_p_reread.log) differing reps"; grep -v amdgpu gpurun_out/r05_p_reread.log | cut -c1-220 | tail -12; ok $rc
RACE_MITIGATE="reread" timeout -k 10 300 python -u tools/race_trace.py 1 30 256 > gpurun_out/r05_p_reread1.log 2>&1; rc=$?
echo "== reread 1 proc exit $rc"; grep -v amdgpu gpurun_out/r05_p_reread1.log | cut -c1-220 | tail -3; ok $rc
