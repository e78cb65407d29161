# Round 5: q6 pass phase timing from the Q6_DIAG_STAMPS build (tools/q6_stamps.py) after the keep-bit
# plane, the spill / prefetch work, the residual codes and the block-maxima trees.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BNN_LIB=$R/abv/stamps/libbnn.so timeout -k 10 300 python tools/q6_stamps.py > gpurun_out/r05_q6_stamps.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r05_q6_stamps.log | tail -24; exit $rc
