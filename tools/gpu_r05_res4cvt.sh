# Residual-plane codes from the FP4 conversion unit: parity (residual decode, hand-off bit-identity,
# z16, keep bits, config-5 step), then A/B against HEAD's build (abv/base: integer residual codes),
# alternating default-bench runs with the bench kernel timers.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp6.py tests/test_gpu_q6_handoff.py tests/test_gpu_z16.py tests/test_gpu_keep_bits.py tests/test_gpu_wide_step.py > gpurun_out/r05_res4cvt_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/r05_res4cvt_tests.log; exit 1; }
tail -2 gpurun_out/r05_res4cvt_tests.log
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export BNN_LIB=$GRAFT_REPO_ROOT/abv/base/libbnn.so; else unset BNN_LIB; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_res4cvt_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_res4cvt_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_res4cvt_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:34]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'q6' in n or 'fp6' in n))"
  done
done
