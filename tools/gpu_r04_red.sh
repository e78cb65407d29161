# Round 4 GPU call: occupancy variants of the BatchNorm reduction passes (RED_OCC / RED_RB /
# HRED_OCC build macros), kernel stats of the bench step in alternation.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
AB_GREP="bn_reduce_k|dz_quant|kernel time" LIBS="tree=distributed-mnist-bnns_amd/lib/libbnn.so r3=ab/r3/libbnn.so h3=ab/h3/libbnn.so rb4=ab/rb4/libbnn.so" bash tools/gpu_r04_ab.sh
