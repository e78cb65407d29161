# popcount conv engine: parity tests, A/B timing, kernel trace; then the uninitialised-memory probe
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_popc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05_i_popc_tests.log 2>&1; rc=$?
echo "POPC tests exit $rc"; grep -E "PASS|FAIL|Error" gpurun_out/r05_i_popc_tests.log | cut -c1-250 | tail -20; ok $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u tools/conv_popc_ab.py 4096 > gpurun_out/r05_i_popc_ab.log 2>&1; rc=$?; cat gpurun_out/r05_i_popc_ab.log | grep -v amdgpu | tail -8; ok $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05_i_prof -o popc -- python3 $R/tools/conv_popc_ab.py 4096 > $R/gpurun_out/r05_i_prof.log 2>&1; rc=$?; echo "PROF exit $rc"; ok $rc
cd $R
timeout -k 10 400 python -u tools/garbage_probe.py cnn config2 mlp > gpurun_out/r05_i_garbage.log 2>&1; rc=$?
echo "GARBAGE exit $rc"; grep -E "DIFF|GARBAGE_PROBE|Error" gpurun_out/r05_i_garbage.log | cut -c1-250 | head -30
