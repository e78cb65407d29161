# Round 4 GPU call: the config-3 MLP (HIP graph) with fc1's s20 hand-off on / off, kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for s in 1 0; do
  BNN_S20=$s bash tools/gpu_stats.sh mlp_s20_$s --config mlp --graph > gpurun_out/mlp_s20_$s.txt 2>&1 || { echo "STATS $s FAIL"; tail -5 gpurun_out/mlp_s20_$s.txt; exit 1; }
  echo "== S20=$s: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_mlp_s20_$s.log)"
  head -22 gpurun_out/mlp_s20_$s.txt | cut -c1-140
done
for s in 1 0; do BNN_S20=$s timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/mlp_g_s20_$s.log 2>&1 && echo "S20=$s bench: $(tail -1 gpurun_out/mlp_g_s20_$s.log | grep -o '"ms_per_step": [0-9.]*')"; done
