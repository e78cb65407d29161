# Round 6, call F: (1) the one-rank RCCL MLP graph-vs-eager difference with the library of call C
# (where the graph test passed) -- a csrc regression or not; (2) the BinCNN stage tracer with
# agent-scope atomic loads on every compact conv reader (BN2_LOADS=2, round 5's instruction form).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BNN_LIB=$R/abv/c_era/libbnn.so timeout -k 10 300 python -u tools/det_rccl_probe.py 3 > gpurun_out/r06_f_det_rccl_c_era.log 2>&1 || { echo DET FAIL; tail -20 gpurun_out/r06_f_det_rccl_c_era.log; exit 1; }
grep -E "^(eager|exchange|graph)" gpurun_out/r06_f_det_rccl_c_era.log
BNN_LIB=$R/abv/bn2_loads2/libbnn.so timeout -k 10 400 python -u tools/race_trace.py 4 30 256 > gpurun_out/r06_f_race_trace_atomic.log 2>&1 || { echo TRACE FAIL; tail -20 gpurun_out/r06_f_race_trace_atomic.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_f_race_trace_atomic.log | cut -c1-220
