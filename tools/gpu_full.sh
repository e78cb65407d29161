# Full GPU session: parity tests, smoke, bench (wide/mlp/cnn), rocprofv3 kernel-trace stats and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the default bench.  Every GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_$TAG.log 2>&1 || { echo PARITY FAIL; tail -30 gpurun_out/parity_$TAG.log; exit 1; }
tail -1 gpurun_out/parity_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_wide_$TAG.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench_wide_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_wide_$TAG.log | cut -c1-400
timeout -k 10 300 python bench.py --config mlp --steps 20 --warmup 3 > gpurun_out/bench_mlp_$TAG.log 2>&1 || { echo BENCH MLP FAIL; tail -30 gpurun_out/bench_mlp_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_mlp_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --config cnn --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cnn_$TAG.log 2>&1 || { echo BENCH CNN FAIL; tail -30 gpurun_out/bench_cnn_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_cnn_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cnn_$TAG -o cnn --output-format csv -- python3 $R/bench.py --config cnn --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_cnn_$TAG.log 2>&1 || { echo PROF CNN FAIL; tail -20 $R/gpurun_out/prof_cnn_$TAG.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo PMC1 FAIL; tail -20 $R/gpurun_out/pmc_fetch_$TAG.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || { echo PMC2 FAIL; tail -20 $R/gpurun_out/pmc_write_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG $R/gpurun_out/pmc_fetch_$TAG $R/gpurun_out/pmc_write_$TAG -name "*.csv"
