# Round 4 GPU call: fc1's compact output (s20) -- its bit-identity tests, the config-5 step parity
# and the other compact-form tests, then kernel stats of the bench step with the hand-off on / off
# (BNN_S20), twice in alternation.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s20.py tests/test_gpu_wide_step.py tests/test_gpu_z16.py tests/test_gpu_net_configs.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04_s20_tests.log 2>&1
rc=$?; echo "S20 TESTS EXIT $rc"; grep -E "PASS|FAIL|Error|error|config 5" gpurun_out/r04_s20_tests.log | cut -c1-300 | tail -40
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for s in 1 0; do
    BNN_S20=$s bash tools/gpu_stats.sh s20_${s}_$round > gpurun_out/s20_${s}_$round.txt 2>&1 || { echo "STATS $s FAIL"; tail -5 gpurun_out/s20_${s}_$round.txt; exit 1; }
    echo "== S20=$s round $round: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_s20_${s}_$round.log)"
    grep -E "kernel time|gemm_i8_v2_k<1, 1|bn_reduce_k<2|bn_dz_quant|bn_apply_pack_fp4_k<[02]" gpurun_out/s20_${s}_$round.txt | cut -c1-130
  done
done
# the one-input-channel filter-gradient kernel: its tests, then BinCNN kernel stats on / off
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "conv" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_c1f_tests.log 2>&1
rc=$?; echo "C1F TESTS EXIT $rc"; tail -3 gpurun_out/r04_c1f_tests.log
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for s in 1 0; do
    BNN_CONV_C1F=$s bash tools/gpu_stats.sh c1f_${s}_$round --config cnn > gpurun_out/c1f_${s}_$round.txt 2>&1 || { echo "CNN STATS $s FAIL"; tail -5 gpurun_out/c1f_${s}_$round.txt; exit 1; }
    echo "== C1F=$s round $round: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_c1f_${s}_$round.log)"
    grep -E "kernel time|conv_bwd_filter" gpurun_out/c1f_${s}_$round.txt | cut -c1-130
  done
done
