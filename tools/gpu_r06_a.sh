# Round 6, first call: the GPU suite (part A incl. the new DDP-around-drop-in test), smoke, the
# default bench line, the dropout accuracy seed spread and a rocprofv3 kernel
# summary of the drop-in path at config 5.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp_dropin.py -m gpu -v -s -rf --timeout 200 --timeout-method thread > gpurun_out/r06_a_ddp_dropin.log 2>&1; rc=$?
echo "DDP exit $rc"; grep -E "passed|failed|\[org\]|\[frozen\]" gpurun_out/r06_a_ddp_dropin.log | tail -12; grep -E "^E |Error" gpurun_out/r06_a_ddp_dropin.log | cut -c1-300 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread $IGN --deselect tests/test_gpu_ddp_dropin.py > gpurun_out/r06_a_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_a_gpu_tests_a.log | tail -2; grep -E "^FAILED|Error" gpurun_out/r06_a_gpu_tests_a.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06_a_smoke.log 2>&1 || { echo SMOKE FAIL; tail -5 gpurun_out/r06_a_smoke.log; exit 1; }
tail -1 gpurun_out/r06_a_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r06_a_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r06_a_bench.log; exit 1; }
tail -1 gpurun_out/r06_a_bench.log | cut -c1-400
timeout -k 10 300 python -u tools/dropout_seed_spread.py 8 > gpurun_out/r06_a_dropout_spread.log 2>&1 || { echo SPREAD FAIL; tail -5 gpurun_out/r06_a_dropout_spread.log; exit 1; }
cat gpurun_out/r06_a_dropout_spread.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06_dropin -o run --output-format csv -- python3 $R/bench.py --dropin --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing > $R/gpurun_out/r06_a_dropin_prof.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/r06_a_dropin_prof.log; exit 1; }
tail -1 $R/gpurun_out/r06_a_dropin_prof.log | cut -c1-300
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06_dropin -name 'run_kernel_stats.csv' | head -1) 7 40 > $R/gpurun_out/r06_a_dropin_stats.txt
head -30 $R/gpurun_out/r06_a_dropin_stats.txt | cut -c1-170
