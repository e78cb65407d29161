# forward-only device-scope compact loads: contention trace + BinCNN step; config 2 exchange diagnosis
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 300 python -u tools/race_trace.py 4 40 256 > gpurun_out/r05_race_trace_fwdcoh.log 2>&1; rc=$?
echo "== fwd-coherent exit $rc: $(grep -c 'first difference' gpurun_out/r05_race_trace_fwdcoh.log) differing reps"; grep -v amdgpu gpurun_out/r05_race_trace_fwdcoh.log | cut -c1-160 | tail -4; ok $rc
for v in default plain; do
  if [ $v = plain ]; then export BNN_LIB=$R/abv/plain/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 200 python -u bench.py --config cnn --steps 100 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_x_cnn_$v.log 2>&1; rc=$?
  echo "== $v cnn bench exit $rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05_x_cnn_$v.log; ok $rc
done
unset BNN_LIB
for o in "" "direct_write=0" "broadcast_buffers=0"; do
  DIAG_EXCHANGE="$o" timeout -k 10 200 python -u tools/ddp_config2_diag.py 3 > gpurun_out/r05_x_c2_$o.log 2>&1; rc=$?
  echo "== options [$o] exit $rc"; grep -v amdgpu "gpurun_out/r05_x_c2_$o.log" | grep -v "^\[" | cut -c1-230 | tail -14; ok $rc
done
