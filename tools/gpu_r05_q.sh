# (1) the kernel-level probe with the processes overlapping for 20 s; (2) the model trace with the
# compact BatchNorm2d input read by device-scope loads (diagnostic build) against the default build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 200 python -u tools/race_cnn_kernels.py 4 50 256 20 > gpurun_out/r05_q_rk.log 2>&1; rc=$?; echo "RK exit $rc"; grep -v amdgpu gpurun_out/r05_q_rk.log | tail -16; ok $rc
BNN_LIB=$R/abv/coh/libbnn.so timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_q_coh.log 2>&1; rc=$?
echo "== coherent loads exit $rc: $(grep -c 'first difference' gpurun_out/r05_q_coh.log) differing reps"; grep -v amdgpu gpurun_out/r05_q_coh.log | cut -c1-200 | tail -4; ok $rc
timeout -k 10 300 python -u tools/race_trace.py 4 30 256 > gpurun_out/r05_q_def.log 2>&1; rc=$?
echo "== default exit $rc: $(grep -c 'first difference' gpurun_out/r05_q_def.log) differing reps"; grep -v amdgpu gpurun_out/r05_q_def.log | cut -c1-200 | tail -4; ok $rc
