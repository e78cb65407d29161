# Round-6 final artifacts, second pass (HEAD after the conv backward-data tap loop, the drop-in BatchNorm1d hand-off and the DDP org-bn case): the whole GPU suite (A + the long whole-step tests), smoke(), the
# one-rank RCCL probe, small-config lines (BinCNN eager / graph / exchange, MLP config 3, the published
# small config), the default bench line (with the drop-in comparators), rocprofv3 kernel stats +
# FETCH / WRITE traffic of the wide step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_final2_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_final2_gpu_tests_a.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/r06_final2_gpu_tests_a.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/r06_final2_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r06_final2_gpu_tests_b.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/r06_final2_gpu_tests_b.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r06_final2_smoke.log 2>&1 || { echo SMOKE FAIL; tail -5 gpurun_out/r06_final2_smoke.log; exit 1; }
tail -1 gpurun_out/r06_final2_smoke.log
timeout -k 10 300 python -u tools/det_rccl_probe.py 3 > gpurun_out/r06_final2_det_rccl.log 2>&1 || { echo DET FAIL; grep -v "^frame" gpurun_out/r06_final2_det_rccl.log | grep -E "rror" | head -3; }
grep -E "^(eager|exchange|graph)" gpurun_out/r06_final2_det_rccl.log
for c in "cnn" "cnn --graph" "cnn --exchange" "cnn --graph --exchange" "mlp" "mlp --graph" "small" "small --graph"; do
  tag=$(echo $c | tr -d ' -'); timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_final2_bench_$tag.log 2>&1 || { echo BENCH $c FAIL; tail -5 gpurun_out/r06_final2_bench_$tag.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/r06_final2_bench_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 500 python bench.py > gpurun_out/r06_final2_bench_wide.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r06_final2_bench_wide.log; exit 1; }
tail -1 gpurun_out/r06_final2_bench_wide.log | cut -c1-200
TAG=r06f2 bash tools/gpu_profile.sh > gpurun_out/r06_final2_prof.txt 2>&1 || { echo PROF FAIL; tail gpurun_out/r06_final2_prof.txt; exit 1; }
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r06f2 --write gpurun_out/pmc_write_r06f2 --out gpurun_out/r06f2_pmc_traffic.json || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r06f2/wide_kernel_stats.csv 7 30 > gpurun_out/r06_final2_stats.txt || exit 1
head -14 gpurun_out/r06_final2_stats.txt | cut -c1-150
