# Round 6, call E: where the remaining nondeterminism is.  (1) one process, no other GPU work: the
# one-rank RCCL MLP step repeated eagerly, with the exchange, and graph-replayed; (2) the BinCNN
# stage tracer (4 processes) with the default build (sc1 buffer loads on every compact conv reader)
# and with agent-scope atomic loads on every reader (BN2_LOADS=2).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/det_rccl_probe.py 6 > gpurun_out/r06_e_det_rccl.log 2>&1 || { echo DET FAIL; tail -20 gpurun_out/r06_e_det_rccl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_e_det_rccl.log
timeout -k 10 400 python -u tools/race_trace.py 4 30 256 > gpurun_out/r06_e_race_trace_sc1buf.log 2>&1 || { echo TRACE FAIL; tail -20 gpurun_out/r06_e_race_trace_sc1buf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_e_race_trace_sc1buf.log | cut -c1-220
BNN_LIB=$R/ab/bn2_loads2/libbnn.so timeout -k 10 400 python -u tools/race_trace.py 4 30 256 > gpurun_out/r06_e_race_trace_atomic.log 2>&1 || { echo TRACE2 FAIL; tail -20 gpurun_out/r06_e_race_trace_atomic.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_e_race_trace_atomic.log | cut -c1-220
