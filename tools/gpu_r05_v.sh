# device-scope compact loads (default) vs plain: contention trace, BinCNN step; then the
# data-parallel GPU tests and the CNN parity tests on the default build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 300 python -u tools/race_trace.py 4 40 256 > gpurun_out/r05_race_trace_default.log 2>&1; rc=$?
echo "== default exit $rc: $(grep -c 'first difference' gpurun_out/r05_race_trace_default.log) differing reps"; grep -v amdgpu gpurun_out/r05_race_trace_default.log | cut -c1-160 | tail -4; ok $rc
BNN_LIB=$R/abv/plain/libbnn.so timeout -k 10 300 python -u tools/race_trace.py 4 40 256 > gpurun_out/r05_race_trace_plain.log 2>&1; rc=$?
echo "== plain exit $rc: $(grep -c 'first difference' gpurun_out/r05_race_trace_plain.log) differing reps"; ok $rc
for v in default plain; do
  if [ $v = plain ]; then export BNN_LIB=$R/abv/plain/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 200 python -u bench.py --config cnn --steps 100 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_v_cnn_$v.log 2>&1; rc=$?
  echo "== $v cnn bench exit $rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05_v_cnn_$v.log; ok $rc
done
unset BNN_LIB
timeout -k 10 500 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_cnn_parity.py tests/test_gpu_rccl.py -v --timeout 300 --timeout-method thread > gpurun_out/r05_v_tests.log 2>&1; rc=$?
echo "TESTS exit $rc"; grep -E "PASS|FAIL|AssertionError: \(" gpurun_out/r05_v_tests.log | cut -c1-200 | tail -16
