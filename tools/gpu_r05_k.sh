# localise the contention-only BinCNN nondeterminism stage by stage
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 300 python -u tools/race_cnn_kernels.py 1 100 256 > gpurun_out/r05_k_rk1.log 2>&1; rc=$?; echo "RK1 exit $rc"; grep -v amdgpu gpurun_out/r05_k_rk1.log | tail -20; ok $rc
timeout -k 10 300 python -u tools/race_cnn_kernels.py 4 100 256 > gpurun_out/r05_k_rk4.log 2>&1; rc=$?; echo "RK4 exit $rc"; grep -v amdgpu gpurun_out/r05_k_rk4.log | tail -40; ok $rc
timeout -k 10 300 python -u tools/race_cnn_kernels.py 4 60 4096 > gpurun_out/r05_k_rk4b.log 2>&1; rc=$?; echo "RK4b exit $rc"; grep -v amdgpu gpurun_out/r05_k_rk4b.log | tail -40; ok $rc
