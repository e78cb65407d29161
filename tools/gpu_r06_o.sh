# Round 6, call O: the drop-in BatchNorm1d with the FP6 digit hand-off on (dx still written, digits
# keyed to it): its tests, the DDP drop-in tests, and the wide drop-in step with it.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bn_dropin.py \
  tests/test_gpu_q6_handoff.py tests/test_gpu_ddp_dropin.py > gpurun_out/r06_o_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_o_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_o_gpu_tests.log | tail -1
timeout -k 10 400 python bench.py --dropin --dropin-bn --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch > gpurun_out/r06_o_bench_dropin_bn.log 2>&1 || { echo BENCH FAIL; tail -5 gpurun_out/r06_o_bench_dropin_bn.log; exit 1; }
tail -1 gpurun_out/r06_o_bench_dropin_bn.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06o_dropinbn -o run --output-format csv -- python3 $R/bench.py --dropin --dropin-bn --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_o_dropinbn_prof.log 2>&1 || { echo PROF FAIL; tail -5 $R/gpurun_out/r06_o_dropinbn_prof.log; exit 1; }
python3 $R/tools/dropin_breakdown.py $(find $R/gpurun_out/prof_r06o_dropinbn -name 'run_kernel_stats.csv' | head -1) 7 > $R/gpurun_out/r06_o_dropinbn_breakdown.txt
head -20 $R/gpurun_out/r06_o_dropinbn_breakdown.txt | cut -c1-150
