# Full GPU test suite, then bench lines (wide default + the given extra configs) and kernel stats
# of the MLP config.  bash tools/gpu_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; tail -2 gpurun_out/gpu_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
summ() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'].get('model'), d['value'], d['ms_per_step']); [print('  ', k, v['avg_us'], v['launches_per_step']) for k,v in list(d['kernels'].items())[:8]]"; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gpu-torch > gpurun_out/bench_wide.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/bench_wide.log; exit 1; }
summ gpurun_out/bench_wide.log
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > gpurun_out/bench_mlp.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/bench_mlp.log; exit 1; }
tail -1 gpurun_out/bench_mlp.log | cut -c1-200
bash tools/gpu_stats.sh mlp --config mlp > gpurun_out/stats_mlp.txt || exit 1
head -14 gpurun_out/stats_mlp.txt | cut -c1-160
