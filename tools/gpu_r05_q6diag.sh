# Where the quantising BatchNorm passes spend their time (timing-only builds, wrong results):
# in-tree (base) vs abv/noquant (no FP6 quantisation) vs abv/nocsum (no column sums) vs
# BNN_FP6_RES=0 (no residual plane), alternating default-bench runs, bench kernel timers.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2; do
  for v in base noquant nocsum nores; do
    unset BNN_LIB BNN_FP6_RES
    case $v in noquant|nocsum) export BNN_LIB=$GRAFT_REPO_ROOT/abv/$v/libbnn.so;; nores) export BNN_FP6_RES=0;; esac
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_q6diag_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_q6diag_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_q6diag_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v r$r', d['ms_per_step'], ' | '.join(f'{n[:34]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'q6' in n or 'i8cols' in n or 'fp6' in n))"
  done
done
