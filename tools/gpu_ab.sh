# A/B of two libbnn builds on one box: ab/libbnn_a.so (A) against the in-tree library (B),
# alternating default-bench runs (kernel timers on), ROUNDS rounds.  bash tools/gpu_ab.sh [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for v in A B; do
    if [ $v = A ]; then export BNN_LIB=$GRAFT_REPO_ROOT/ab/libbnn_a.so; else unset BNN_LIB; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gpu-torch ${BENCH_ARGS} > gpurun_out/ab_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/ab_$v$r.log; exit 1; }
    tail -1 gpurun_out/ab_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' '.join(f'{n[:14]}={v[\"avg_us\"]:.0f}' for n,v in list(k.items())[:7]))"
  done
done
