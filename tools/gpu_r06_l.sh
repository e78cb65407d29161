# Round 6, call L: bnn_amd.nn.BatchNorm1d (torch's module on libbnn's passes) -- its tests and the
# wide drop-in step with it (rocprof split); BinCNN graph-step kernel stats; effective clock of the
# FP6 GEMM launches in the fused wide step vs the drop-in path (GRBM_GUI_ACTIVE passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bn_dropin.py \
  > gpurun_out/r06_l_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_l_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_l_gpu_tests.log | tail -1
timeout -k 10 400 python bench.py --dropin --dropin-bn --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch > gpurun_out/r06_l_bench_dropin_bn.log 2>&1 || { echo BENCH FAIL; tail -5 gpurun_out/r06_l_bench_dropin_bn.log; exit 1; }
tail -1 gpurun_out/r06_l_bench_dropin_bn.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06l_dropinbn -o run --output-format csv -- python3 $R/bench.py --dropin --dropin-bn --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_l_dropinbn_prof.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_l_dropinbn_prof.log; exit 1; }
python3 $R/tools/dropin_breakdown.py $(find $R/gpurun_out/prof_r06l_dropinbn -name 'run_kernel_stats.csv' | head -1) 7 > $R/gpurun_out/r06_l_dropinbn_breakdown.txt
head -32 $R/gpurun_out/r06_l_dropinbn_breakdown.txt | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06l_cnng -o cnng --output-format csv -- python3 $R/bench.py --config cnn --graph --steps 100 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_l_cnng_prof.log 2>&1 || { echo PROF CNNG FAIL; tail -5 $R/gpurun_out/r06_l_cnng_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06l_cnng -name 'cnng_kernel_stats.csv' | head -1) 105 40 > $R/gpurun_out/r06_l_cnng_stats.txt
head -24 $R/gpurun_out/r06_l_cnng_stats.txt | cut -c1-150
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_clk_wide -o wide --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_l_clk_wide.log 2>&1 || { echo PMC WIDE FAIL; tail -5 $R/gpurun_out/r06_l_clk_wide.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_clk_dropin -o dropin --output-format csv -- python3 $R/bench.py --dropin --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_l_clk_dropin.log 2>&1 || { echo PMC DROPIN FAIL; tail -5 $R/gpurun_out/r06_l_clk_dropin.log; exit 1; }
python3 $R/tools/clk_table.py $R/gpurun_out/pmc_clk_wide $R/gpurun_out/pmc_clk_dropin gemm_ > $R/gpurun_out/r06_l_clk_table.txt
cat $R/gpurun_out/r06_l_clk_table.txt
