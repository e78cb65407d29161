# popcount wpack fix + A/B; run-to-run determinism under contention (1 and 2 processes)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_popc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_j_popc_tests.log 2>&1; rc=$?
echo "POPC tests exit $rc"; tail -3 gpurun_out/r05_j_popc_tests.log; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u tools/conv_popc_ab.py 4096 > gpurun_out/r05_j_popc_ab.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r05_j_popc_ab.log | tail -8; ok $rc
timeout -k 10 300 python -u tools/race_probe.py 1 20 cnn config2 mlp > gpurun_out/r05_j_race1.log 2>&1; rc=$?; echo "RACE1 exit $rc"; grep -v amdgpu gpurun_out/r05_j_race1.log | tail -20; ok $rc
timeout -k 10 400 python -u tools/race_probe.py 2 20 cnn config2 mlp > gpurun_out/r05_j_race2.log 2>&1; rc=$?; echo "RACE2 exit $rc"; grep -v amdgpu gpurun_out/r05_j_race2.log | tail -40; ok $rc
