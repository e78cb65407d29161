# Round 4: q6 timing-only build without the column sums (ncs) against the tree (C).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
AB_GREP="q6_k" LIBS="C=ab/C/libbnn.so ncs=ab/ncs/libbnn.so" bash tools/gpu_r04_ab.sh
