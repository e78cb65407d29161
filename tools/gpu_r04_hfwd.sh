# Round 4: the head's forward (bn_head_fwd_k<10, z16>) compiled for 3 waves per SIMD (-DHFWD_OCC=3:
# 135 VGPRs, no spills) against HEAD's 4 (128 VGPRs, 5 spilled) -- kernel stats of the bench step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
AB_GREP="bn_head_fwd" LIBS="O=ab/O/libbnn.so f3=ab/f3/libbnn.so" bash tools/gpu_r04_ab.sh
