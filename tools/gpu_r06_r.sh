# Round 6, call R: BinCNN eager step, previous build vs HEAD in alternating order (is call Q's slower
# eager line for HEAD real?), 3 rounds of 300 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in pre head; do
    if [ $lib = pre ]; then export BNN_LIB=$R/abv/preconv/libbnn.so; else unset BNN_LIB; fi
    timeout -k 10 300 python bench.py --config cnn --steps 300 --warmup 20 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_r_cnn_${lib}_$rep.log 2>&1 || { echo BENCH FAIL; tail -5 gpurun_out/r06_r_cnn_${lib}_$rep.log; exit 1; }
    echo "cnn_${lib}_$rep: $(tail -1 gpurun_out/r06_r_cnn_${lib}_$rep.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
