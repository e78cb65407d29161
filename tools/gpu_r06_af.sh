# Round 6, call AF: the binarized weights' Adam + pack launches on side streams (optim.ADAM_STREAMS,
# env BNN_ADAM_STREAMS; HEAD default 2) -- GPU suites A + B and smoke on the default, then graph
# steps (config 3, BinCNN, small net) and wide steps interleaved with BNN_ADAM_STREAMS=0.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_af_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_af_gpu_tests_a.log | tail -1; grep -E "^FAILED" gpurun_out/r06_af_gpu_tests_a.log | head
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -q -rf --timeout 600 --timeout-method thread > gpurun_out/r06_af_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r06_af_gpu_tests_b.log | tail -1; grep -E "^FAILED" gpurun_out/r06_af_gpu_tests_b.log | head
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06_af_smoke.log 2>&1 || { echo SMOKE FAIL; tail -5 gpurun_out/r06_af_smoke.log; exit 1; }
tail -1 gpurun_out/r06_af_smoke.log
for rep in 1 2; do
  for cfg in mlp cnn small; do
    for ns in 2 0; do
      tag=${cfg}g_s${ns}_$rep
      BNN_ADAM_STREAMS=$ns timeout -k 10 300 python bench.py --config $cfg --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_af_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_af_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_af_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
  for ns in 2 0; do
    tag=wide_s${ns}_$rep
    BNN_ADAM_STREAMS=$ns timeout -k 10 400 python bench.py --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_af_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_af_$tag.log; exit 1; }
    echo "$tag: $(tail -1 gpurun_out/r06_af_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
