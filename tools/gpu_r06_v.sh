# Round 6, call V: raster group (tile rows per group, tile6_of) of the FP6 half-tile dX form.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u tools/fp6_half_ab.py "0:0 1:0 1:0:2 1:0:4 1:0:8 1:0:16 1:0:32" 4 3 > gpurun_out/r06_v_fp6_group.log 2>&1 || { echo AB FAIL; tail -10 gpurun_out/r06_v_fp6_group.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_v_fp6_group.log
