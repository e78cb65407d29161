# A/B on one box: abv/base/libbnn.so (HEAD: dY4 rows loaded at each q6 sub-tile top) against the in-tree
# library (dY4 rows and keep words prefetched with the x loads), alternating default-bench runs with
# the bench kernel timers, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export BNN_LIB=$GRAFT_REPO_ROOT/abv/base/libbnn.so; else unset BNN_LIB; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_d4pref_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_d4pref_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_d4pref_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:40]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'q6' in n or 'head' in n or 'fp6' in n))"
  done
done
