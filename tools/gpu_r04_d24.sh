# Round 4 GPU call: one-add/one-xor int8 digit packing (digits24) + alignbit s20 decode -- the
# bit-identity tests, then kernel stats of the bench step with fc1's s20 hand-off on / off.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s20.py tests/test_gpu_parity.py tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -k "s20 or quant or i8c or digit or config5 or gemm_i8" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04_d24_tests.log 2>&1
rc=$?; echo "D24 TESTS EXIT $rc"; grep -cE "PASSED" gpurun_out/r04_d24_tests.log; grep -E "FAIL|Error|config 5" gpurun_out/r04_d24_tests.log | cut -c1-300 | tail -20
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for s in 1 0; do
    BNN_S20=$s bash tools/gpu_stats.sh d24_${s}_$round > gpurun_out/d24_${s}_$round.txt 2>&1 || { echo "STATS $s FAIL"; tail -5 gpurun_out/d24_${s}_$round.txt; exit 1; }
    echo "== S20=$s round $round: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_d24_${s}_$round.log)"
    grep -E "kernel time|gemm_i8_v2_k<1, 1|bn_reduce_k<2|bn_dz_quant|bn_apply_pack_fp4_k<[02]|gemm_i8_v2_k<3" gpurun_out/d24_${s}_$round.txt | cut -c1-130
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "conv1_filter or full_batch" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_c1f2_tests.log 2>&1
rc=$?; echo "C1F TESTS EXIT $rc"; tail -2 gpurun_out/r04_c1f2_tests.log
[ $rc -eq 0 ] || exit $rc
for s in 1 0; do
  BNN_CONV_C1F=$s bash tools/gpu_stats.sh c1fb_${s} --config cnn > gpurun_out/c1fb_${s}.txt 2>&1 || { echo "CNN STATS $s FAIL"; tail -5 gpurun_out/c1fb_${s}.txt; exit 1; }
  echo "== C1F=$s: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_c1fb_${s}.log)"
  grep -E "kernel time|conv_bwd_filter" gpurun_out/c1fb_${s}.txt | cut -c1-130
done
# SQ PMC passes over the bench step's kernels (instruction mix / busy / wait per kernel)
TAG=r04d24 bash tools/gpu_r04_prof.sh > gpurun_out/r04d24_prof.txt 2>&1; echo "PROF EXIT $?"; tail -3 gpurun_out/r04d24_prof.txt
grep -E "dz_quant|q6_k|head|reduce_k<2|apply_pack" gpurun_out/pmc_r04d24_all.txt | cut -c1-250
