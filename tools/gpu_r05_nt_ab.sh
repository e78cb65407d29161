# Non-temporal record stores in the quantising passes: plain stores (abv/plain = HEAD), NT q6 digit
# records only (abv/q6nt), NT q6 records + int8 column digits (in-tree); parity tests of the q6 / s20
# paths on the in-tree library, then default-bench runs with the kernel timers, alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_q6_handoff.py tests/test_gpu_s20.py tests/test_gpu_z16.py > gpurun_out/r05_nt_tests.log 2>&1 \
  || { echo "TESTS FAIL"; tail -30 gpurun_out/r05_nt_tests.log; exit 1; }
tail -2 gpurun_out/r05_nt_tests.log
for r in 1 2 3; do
  for v in plain q6nt new; do
    if [ $v = new ]; then unset BNN_LIB; else export BNN_LIB=$GRAFT_REPO_ROOT/abv/$v/libbnn.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_nt_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_nt_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_nt_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:26]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if v['avg_us'] > 900))"
  done
done
