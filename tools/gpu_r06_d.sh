# Round 6, call D: sc1 buffer loads for every compact conv reader, residual plane from 8192 rows,
# ToTensor recognition incl. the GPU's reciprocal division: GPU suite (A + long), small-config
# benches (BinCNN eager / graph, MLP config 3 graph), the default bench line, drop-in profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_d_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_d_gpu_tests_a.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/r06_d_gpu_tests_a.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/r06_d_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r06_d_gpu_tests_b.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/r06_d_gpu_tests_b.log | cut -c1-250 | head -12; grep -E "Net r=3 batch|BinCNN step" gpurun_out/r06_d_gpu_tests_b.log | cut -c1-200
case $rc in 0|1) ;; *) exit $rc;; esac
for c in "cnn" "cnn --graph" "mlp --graph"; do
  tag=$(echo $c | tr -d ' -'); timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_d_bench_$tag.log 2>&1 || { echo BENCH $c FAIL; tail -5 gpurun_out/r06_d_bench_$tag.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/r06_d_bench_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 python bench.py > gpurun_out/r06_d_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r06_d_bench.log; exit 1; }
tail -1 gpurun_out/r06_d_bench.log | cut -c1-160; tail -1 gpurun_out/r06_d_bench.log | grep -o '"dropin": {[^}]*}' | cut -c1-120
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06d_dropin -o run --output-format csv -- python3 $R/bench.py --dropin --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_d_dropin_prof.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/r06_d_dropin_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06d_dropin -name 'run_kernel_stats.csv' | head -1) 7 40 > $R/gpurun_out/r06_d_dropin_stats.txt
head -24 $R/gpurun_out/r06_d_dropin_stats.txt | cut -c1-170
