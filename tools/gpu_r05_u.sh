# the BatchNorm2d forward sequence: host sync between its kernels / device-scope statistics loads
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for v in sync cohstats; do
  BNN_LIB=$R/abv/$v/libbnn.so timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_u_$v.log 2>&1; rc=$?
  echo "== variant [$v] exit $rc: $(grep -c 'first difference' gpurun_out/r05_u_$v.log) differing reps"; grep -v amdgpu "gpurun_out/r05_u_$v.log" | cut -c1-200 | tail -3; ok $rc
done
