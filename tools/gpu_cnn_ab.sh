# CNN kernel A/B: conv parity tests, then rocprofv3 kernel stats of the BinCNN bench with
# ab/libbnn_a.so (A) and the in-tree library (B).  bash tools/gpu_cnn_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or cnn" > gpurun_out/cnn_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/cnn_tests.log; exit 1; }
tail -1 gpurun_out/cnn_tests.log
for v in A B; do
  if [ $v = A ]; then export BNN_LIB=$GRAFT_REPO_ROOT/ab/libbnn_a.so; else unset BNN_LIB; fi
  rm -rf gpurun_out/prof_cnn_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cnn_$v -o run --output-format csv -- python bench.py --config cnn --steps 20 --warmup 3 --no-cpu-baseline --no-gpu-torch > gpurun_out/bench_cnn_$v.log 2>&1 || { echo "BENCH $v FAIL"; tail -5 gpurun_out/bench_cnn_$v.log; exit 1; }
  grep "^{" gpurun_out/bench_cnn_$v.log | cut -c1-150
  f=$(find gpurun_out/prof_cnn_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:9]:
    print(f"   {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
