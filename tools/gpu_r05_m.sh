# stage-by-stage trace of the contention-only BinCNN nondeterminism (compact conv outputs on)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for f in "" "C1BN=0"; do
  RACE_PROBE_FLAGS="$f" timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_m_trace_$f.log 2>&1; rc=$?
  echo "== flags [$f] exit $rc"; grep -v amdgpu "gpurun_out/r05_m_trace_$f.log" | cut -c1-330 | tail -30; ok $rc
done
