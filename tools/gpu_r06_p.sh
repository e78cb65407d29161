# Round 6, call P: SQ counters of the BinCNN step's conv backward kernels (what bounds them).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
BENCH_ARGS="--config cnn --no-dropin" bash tools/gpu_pmc_bench.sh r06p_cnn conv_ > gpurun_out/r06_p_pmc_cnn.txt 2>&1 || { echo PMC FAIL; tail -20 gpurun_out/r06_p_pmc_cnn.txt; exit 1; }
cat gpurun_out/r06_p_pmc_cnn.txt | cut -c1-150
