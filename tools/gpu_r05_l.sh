# which BinCNN fusion carries the contention-only nondeterminism
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for f in "" "C1BN=0" "ZQ=0" "C1BN=0,ZQ=0"; do
  RACE_PROBE_FLAGS="$f" timeout -k 10 300 python -u tools/race_probe.py 4 30 cnn > gpurun_out/r05_l_race_$f.log 2>&1; rc=$?
  echo "== flags [$f] exit $rc"; grep -v amdgpu "gpurun_out/r05_l_race_$f.log" | tail -16; ok $rc
done
