# Round 4: the head's q6 pass compiled for 2 waves per SIMD (-DQ6_HEAD_OCC=2: 178 VGPRs, no spills)
# against HEAD's 3 (168 VGPRs, 5 spilled) -- kernel stats of the bench step in alternation.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
AB_GREP="q6_k" LIBS="O=ab/O/libbnn.so h2=ab/h2/libbnn.so" bash tools/gpu_r04_ab.sh
