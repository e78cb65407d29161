# Round 6, call K: rocprofv3 kernel stats of the BinCNN HIP-graph step (what the atomic compact
# reads cost, what else is left); GRBM_GUI_ACTIVE (GPU clock cycles) per FP6 GEMM launch in the
# fused wide step and in the drop-in path (is the drop-in's slower dX a clock difference?).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06k_cnng -o cnng --output-format csv -- python3 $R/bench.py --config cnn --graph --steps 100 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_k_cnng_prof.log 2>&1 || { echo PROF CNNG FAIL; tail -5 $R/gpurun_out/r06_k_cnng_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06k_cnng -name 'cnng_kernel_stats.csv' | head -1) 105 40 > $R/gpurun_out/r06_k_cnng_stats.txt
head -26 $R/gpurun_out/r06_k_cnng_stats.txt | cut -c1-150
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_clk_wide -o wide --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_k_clk_wide.log 2>&1 || { echo PMC WIDE FAIL; tail -5 $R/gpurun_out/r06_k_clk_wide.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_clk_dropin -o dropin --output-format csv -- python3 $R/bench.py --dropin --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_k_clk_dropin.log 2>&1 || { echo PMC DROPIN FAIL; tail -5 $R/gpurun_out/r06_k_clk_dropin.log; exit 1; }
python3 $R/tools/clk_table.py $R/gpurun_out/pmc_clk_wide $R/gpurun_out/pmc_clk_dropin gemm_ > $R/gpurun_out/r06_k_clk_table.txt
cat $R/gpurun_out/r06_k_clk_table.txt
