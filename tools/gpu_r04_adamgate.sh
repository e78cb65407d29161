# Round 4: the 256 x 256-tile Adam kernel only for grids of >= 512 whole tiles -- the Adam /
# training tests, then the config-3 MLP (HIP graph and eager) with the gate (tree) and with the big
# tile forced (BNN_ADAM_TILE256=2), kernel stats of the graph runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_adamgate_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04_adamgate_tests.log; [ $rc = 0 ] || exit 1
for t in 1 2; do
  BNN_ADAM_TILE256=$t bash tools/gpu_stats.sh mlp_t$t --config mlp --graph > gpurun_out/mlp_t$t.txt 2>&1 || { echo "STATS $t FAIL"; tail -5 gpurun_out/mlp_t$t.txt; exit 1; }
  echo "== TILE256=$t: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_mlp_t$t.log)"
  grep -E "adam|sign_pack|apply_pack" gpurun_out/mlp_t$t.txt | cut -c1-140
done
for t in 1 2; do
  BNN_ADAM_TILE256=$t timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/mlp_g_t$t.log 2>&1 || { echo BENCH FAIL; tail -3 gpurun_out/mlp_g_t$t.log; exit 1; }
  echo "TILE256=$t graph: $(tail -1 gpurun_out/mlp_g_t$t.log | grep -o '"ms_per_step": [0-9.]*')"
  BNN_ADAM_TILE256=$t timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/mlp_e_t$t.log 2>&1 || { echo BENCH FAIL; tail -3 gpurun_out/mlp_e_t$t.log; exit 1; }
  echo "TILE256=$t eager: $(tail -1 gpurun_out/mlp_e_t$t.log | grep -o '"ms_per_step": [0-9.]*')"
done
