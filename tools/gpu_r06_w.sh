# Round 6, call W: what the 256 x 256 apply-pack's transposed (panel) stores cost -- kernel stats of
# the wide step with HEAD and with a timing-only build without those stores (APK_DIAG_NOQT).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for tag in head noqt; do
    BNN_LIB=$R/abv/$tag/libbnn.so bash tools/gpu_stats.sh w_${tag}_$round --no-dropin > gpurun_out/r06_w_${tag}_$round.txt 2>&1 || { echo "AB $tag FAIL"; tail -5 gpurun_out/r06_w_${tag}_$round.txt; exit 1; }
    echo "== $tag round $round"; grep -E "apply_pack_fp4" gpurun_out/r06_w_${tag}_$round.txt | cut -c1-110
  done
done
