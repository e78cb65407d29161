# Round-3 final artifacts: every -m gpu test, smoke(), the default bench line (as the driver runs
# it), CNN / MLP (eager + HIP graph) lines, rocprofv3 kernel-trace stats of the wide step and the
# FETCH/WRITE PMC passes -> per-kernel traffic.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -2 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/final_cnn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/final_mlp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/final_mlp_g.log 2>&1 || exit 1
TAG=r03 bash tools/gpu_profile.sh > gpurun_out/final_prof.txt 2>&1 || { echo PROF FAIL; tail gpurun_out/final_prof.txt; exit 1; }
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r03 --write gpurun_out/pmc_write_r03 --out gpurun_out/r03_pmc_traffic.json || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r03/wide_kernel_stats.csv 7 20 > gpurun_out/final_stats.txt || exit 1
head -12 gpurun_out/final_stats.txt | cut -c1-160
