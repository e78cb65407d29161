# Round 4 GPU call: bank-conflict-free LDS layouts of the bf16x3 conv backward kernels (row pixel
# tiles + 16 (mod 32) pitches in backward data; padded shifted copies in backward filter) -- the
# conv parity tests, BinCNN kernel stats; then the BatchNorm-reduction occupancy A/B of the wide step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cnn_parity.py -k "conv or cnn or CNN" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_conv_tests.log 2>&1
rc=$?; echo "CONV TESTS EXIT $rc"; tail -3 gpurun_out/r04_conv_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  bash tools/gpu_stats.sh cnnlds_$r --config cnn > gpurun_out/cnnlds_$r.txt 2>&1 || { echo "CNN STATS FAIL"; tail -5 gpurun_out/cnnlds_$r.txt; exit 1; }
  echo "== CNN round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_cnnlds_$r.log)"
  head -12 gpurun_out/cnnlds_$r.txt | cut -c1-140
done
bash tools/gpu_r04_red.sh
