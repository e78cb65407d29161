# which mitigation removes the BatchNorm2d-forward nondeterminism under contention
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for m in sync_before sync_after clone_zq zero_ws; do
  RACE_MITIGATE="$m" timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_n_$m.log 2>&1; rc=$?
  echo "== mitigate [$m] exit $rc: $(grep -c 'first difference' gpurun_out/r05_n_$m.log) differing reps"; grep -v amdgpu "gpurun_out/r05_n_$m.log" | cut -c1-200 | tail -4; ok $rc
done
