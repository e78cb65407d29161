# dword-paired int16 conv output stores: compact-output parity, then the contention trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_popc.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "popc or compact or conv" > gpurun_out/r05_s_tests.log 2>&1; rc=$?
echo "TESTS exit $rc"; tail -3 gpurun_out/r05_s_tests.log; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_s_trace.log 2>&1; rc=$?
echo "== paired stores exit $rc: $(grep -c 'first difference' gpurun_out/r05_s_trace.log) differing reps"; grep -v amdgpu gpurun_out/r05_s_trace.log | cut -c1-200 | tail -4; ok $rc
timeout -k 10 200 python -u bench.py --config cnn --steps 50 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_s_cnn.log 2>&1; rc=$?
echo "== cnn bench exit $rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05_s_cnn.log; ok $rc
