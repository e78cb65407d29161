# Round 6, call N: phase-1 row unroll (rows in flight per wave) of the 256 x 256-tile passes
# (bn_apply_pack_fp4_k, adam_pack_fp4_k): 4 (HEAD) vs 8 vs 16, kernel-trace stats of the wide step,
# two alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for round in 1 2; do
  for tag in head apk8 apk16; do
    BNN_LIB=$R/abv/$tag/libbnn.so bash tools/gpu_stats.sh n_${tag}_$round --no-dropin > gpurun_out/r06_n_${tag}_$round.txt 2>&1 || { echo "AB $tag FAIL"; tail -5 gpurun_out/r06_n_${tag}_$round.txt; exit 1; }
    echo "== $tag round $round: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_n_${tag}_$round.log)"
    grep -E "apply_pack_fp4|adam_pack" gpurun_out/r06_n_${tag}_$round.txt | cut -c1-110
  done
done
# the final merges' batched loads: FF_B = 8 (HEAD) vs 16 partials per round (same summation order)
for rep in 1 2; do
  for tag in head ffb16; do
    for c in "mlp --graph" "cnn --graph"; do
      t=$(echo $c | tr -d ' -')_${tag}_$rep
      BNN_LIB=$R/abv/$tag/libbnn.so timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_n_$t.log 2>&1 || { echo BENCH $t FAIL; tail -5 gpurun_out/r06_n_$t.log; exit 1; }
      echo "$t: $(tail -1 gpurun_out/r06_n_$t.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
