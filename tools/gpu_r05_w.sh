# config 2's two-rank exchange: which copy departs from the exact gradient average, and with which options
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
for o in "" "direct_write=0" "broadcast_buffers=0"; do
  DIAG_EXCHANGE="$o" timeout -k 10 200 python -u tools/ddp_config2_diag.py 3 > gpurun_out/r05_w_$o.log 2>&1; rc=$?
  echo "== options [$o] exit $rc"; grep -v amdgpu "gpurun_out/r05_w_$o.log" | grep -v "^\[" | cut -c1-230 | tail -14; ok $rc
done
