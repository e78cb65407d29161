# split the clone mitigation: the int16 sums, the bias, or either with the originals kept alive
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for m in clone_q clone_b clone_zq,keep clone_b,keep; do
  RACE_MITIGATE="$m" timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_o_$m.log 2>&1; rc=$?
  echo "== mitigate [$m] exit $rc: $(grep -c 'first difference' gpurun_out/r05_o_$m.log) differing reps"; grep -v amdgpu "gpurun_out/r05_o_$m.log" | cut -c1-200 | tail -3; ok $rc
done
