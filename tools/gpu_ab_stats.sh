# Kernel-trace stats of the bench step for each library given (A/B timing of a kernel change):
#   bash tools/gpu_ab_stats.sh TAG1=path/to/libbnn.so TAG2=... (bench args in BENCH_ARGS)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  tag=${spec%%=*}; lib=${spec#*=}
  BNN_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_$tag -o ab_$tag --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing $BENCH_ARGS \
    > $R/gpurun_out/ab_$tag.log 2>&1 || { echo "AB $tag FAIL"; tail -5 $R/gpurun_out/ab_$tag.log; exit 1; }
  echo "== $tag: $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/ab_$tag.log)"
  f=$(find $R/gpurun_out/ab_$tag -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/prof_summary.py "$f" 7 ${AB_TOP:-25}
done
