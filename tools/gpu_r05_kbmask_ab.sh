# Head statistics pass: keep bits applied as a sign-extended bit mask (in-tree) against the select
# form (abv/base = HEAD); keep-bit / head parity tests on the in-tree library, then default-bench
# runs with the kernel timers, alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_keep_bits.py tests/test_gpu_head.py > gpurun_out/r05_kbmask_tests.log 2>&1 \
  || { echo "TESTS FAIL"; tail -30 gpurun_out/r05_kbmask_tests.log; exit 1; }
tail -2 gpurun_out/r05_kbmask_tests.log
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export BNN_LIB=$GRAFT_REPO_ROOT/abv/base/libbnn.so; else unset BNN_LIB; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_kbmask_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_kbmask_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_kbmask_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:40]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'head' in n))"
  done
done
