# Quick GPU check: selected test files (TESTS), then the default bench line (BENCH_ARGS).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; tail -3 gpurun_out/quick_tests.log
grep -E "^FAILED|^ERROR|Error" gpurun_out/quick_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gpu-torch ${BENCH_ARGS} > gpurun_out/quick_bench.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/quick_bench.log; exit 1; }
tail -1 gpurun_out/quick_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v['avg_us'], v['launches_per_step']) for k,v in d['kernels'].items()]"
