# q6 block maxima: row maxima by an 8-lane DPP tree + one plain store (no atomics), column maxima
# pre-reduced in registers and across lane groups in the bn2 form -- parity (hand-off bit-identity,
# z16, keep bits, head) then A/B against HEAD's build (abv/base: one LDS atomic per element).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_q6_handoff.py tests/test_gpu_z16.py tests/test_gpu_keep_bits.py tests/test_gpu_head.py tests/test_gpu_fused.py > gpurun_out/r05_maxab_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/r05_maxab_tests.log; exit 1; }
tail -2 gpurun_out/r05_maxab_tests.log
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export BNN_LIB=$GRAFT_REPO_ROOT/abv/base/libbnn.so; else unset BNN_LIB; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_maxab_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_maxab_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_maxab_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:34]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'q6' in n or 'fp6' in n))"
  done
done
