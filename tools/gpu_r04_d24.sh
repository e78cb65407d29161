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
