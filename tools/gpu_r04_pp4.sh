# Round 4: the interleaved FP6 k loop (PP = 4: all fragment reads right after the barrier, the next
# stage's LDS-DMA pieces between the MFMA groups) against the default, dX and dW shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/fp6_diag.py 65536 8192 8192 5 3 7 17 18 > gpurun_out/r04_pp4_dx.log 2>&1 || { echo DX FAIL; tail -5 gpurun_out/r04_pp4_dx.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_pp4_dx.log
timeout -k 10 300 python tools/fp6_diag.py 8192 8192 65536 5 3 7 17 18 > gpurun_out/r04_pp4_dw.log 2>&1 || { echo DW FAIL; tail -5 gpurun_out/r04_pp4_dw.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_pp4_dw.log
