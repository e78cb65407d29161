# Round 4 GPU call: bn_dz_quant_cols_t_k at 2 / 3 (tree) / 4 waves per SIMD, kernel stats of the
# bench step in alternation; then SQ PMC passes over the BinCNN step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_s20.py -k "i8cols" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_occ_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -2 gpurun_out/r04_occ_tests.log
[ $rc -eq 0 ] || exit $rc
AB_GREP="dz_quant|kernel time" LIBS="occ3=distributed-mnist-bnns_amd/lib/libbnn.so occ2=ab/occ2/libbnn.so occ4=ab/occ4/libbnn.so" bash tools/gpu_r04_ab.sh
TAG=r04cnn PMC=1 BENCH_ARGS="--config cnn" bash tools/gpu_r04_prof.sh > gpurun_out/r04cnn_prof.txt 2>&1; echo "PROF EXIT $?"; head -30 gpurun_out/r04cnn_prof.txt | cut -c1-160
