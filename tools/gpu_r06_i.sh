# Round 6, call I (HEAD: atomic compact-conv loads, guarded pixel recognition in graphs): the whole GPU
# suite (A + long), the one-rank RCCL probe, small-config benches, the default bench line, rocprofv3
# kernel stats + FETCH / WRITE PMC passes of the wide step (traffic for the bench's roofline).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LONG="tests/test_gpu_wide_step.py tests/test_gpu_loss_curve.py tests/test_gpu_wide_trace.py tests/test_gpu_cnn_parity.py tests/test_gpu_net_configs.py tests/test_gpu_training.py"
IGN=""; for f in $LONG; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread $IGN > gpurun_out/r06_i_gpu_tests_a.log 2>&1; rc=$?
echo "SUITE A exit $rc"; grep -E "passed|failed" gpurun_out/r06_i_gpu_tests_a.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/r06_i_gpu_tests_a.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest $LONG -m gpu -v -s -rf --timeout 600 --timeout-method thread > gpurun_out/r06_i_gpu_tests_b.log 2>&1; rc=$?
echo "SUITE B exit $rc"; grep -E "passed|failed" gpurun_out/r06_i_gpu_tests_b.log | tail -2; grep -E "^FAILED|^E  " gpurun_out/r06_i_gpu_tests_b.log | cut -c1-250 | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/det_rccl_probe.py 3 > gpurun_out/r06_i_det_rccl.log 2>&1 || { echo DET FAIL; grep -v "^frame" gpurun_out/r06_i_det_rccl.log | grep -E "error|Error" | head -5; }
grep -E "^(eager|exchange|graph)" gpurun_out/r06_i_det_rccl.log
for c in "cnn" "cnn --graph" "cnn --exchange" "cnn --graph --exchange" "mlp --graph"; do
  tag=$(echo $c | tr -d ' -'); timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_i_bench_$tag.log 2>&1 || { echo BENCH $c FAIL; tail -5 gpurun_out/r06_i_bench_$tag.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/r06_i_bench_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 python bench.py > gpurun_out/r06_i_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r06_i_bench.log; exit 1; }
tail -1 gpurun_out/r06_i_bench.log | cut -c1-160
TAG=r06i bash tools/gpu_profile.sh > gpurun_out/r06_i_prof.txt 2>&1 || { echo PROF FAIL; tail gpurun_out/r06_i_prof.txt; exit 1; }
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r06i --write gpurun_out/pmc_write_r06i --out gpurun_out/r06i_pmc_traffic.json || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r06i/wide_kernel_stats.csv 7 24 > gpurun_out/r06_i_stats.txt || exit 1
head -14 gpurun_out/r06_i_stats.txt | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06i_mlpg -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_i_mlpg_prof.log 2>&1 || { echo PROF MLPG FAIL; tail -5 $R/gpurun_out/r06_i_mlpg_prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06i_mlpg -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_i_mlpg_stats.txt
head -30 $R/gpurun_out/r06_i_mlpg_stats.txt | cut -c1-150
