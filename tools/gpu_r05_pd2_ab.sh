# q6 bn2 pass: two-deep prefetch (in-tree library) against HEAD (abv/base) and the workgroup-range
# guard alone (abv/guard, -DQ6_PREFETCH1): parity tests of the q6 paths on the in-tree library, then
# default-bench runs with the kernel timers, alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_q6_handoff.py tests/test_gpu_z16.py tests/test_gpu_keep_bits.py > gpurun_out/r05_pd2_tests.log 2>&1 \
  || { echo "TESTS FAIL"; tail -30 gpurun_out/r05_pd2_tests.log; exit 1; }
tail -2 gpurun_out/r05_pd2_tests.log
for r in 1 2 3; do
  for v in A G B; do
    case $v in A) export BNN_LIB=$GRAFT_REPO_ROOT/abv/base/libbnn.so;; G) export BNN_LIB=$GRAFT_REPO_ROOT/abv/guard/libbnn.so;; B) unset BNN_LIB;; esac
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_pd2_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_pd2_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_pd2_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:40]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'q6' in n or 'head' in n))"
  done
done
