# Round-5 final artifacts, third pass (HEAD after the block-maxima trees), preceded by the same-mask
# loss test of the bench workload: the default bench line, BinCNN / MLP lines (eager + HIP graph), the
# BinCNN through the exchange (eager and graph-captured), rocprofv3 kernel-trace stats of the wide step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu "tests/test_gpu_wide_step.py::test_wide_bench_loss_same_masks" > gpurun_out/r05_same_masks.log 2>&1; echo "SAME-MASK TEST exit $?"; tail -6 gpurun_out/r05_same_masks.log | cut -c1-400
timeout -k 10 400 python bench.py > gpurun_out/r05_final3_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r05_final3_bench.log; exit 1; }
tail -1 gpurun_out/r05_final3_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final3_cnn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --graph --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final3_cnn_g.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --exchange --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final3_cnn_x.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --graph --exchange --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final3_cnn_gx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/r05_final3_mlp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final3_mlp_g.log 2>&1 || exit 1
for f in cnn cnn_g cnn_x cnn_gx mlp mlp_g; do echo "$f: $(tail -1 gpurun_out/r05_final3_$f.log | grep -o '"ms_per_step": [0-9.]*')"; done
TAG=r05c bash tools/gpu_profile.sh > gpurun_out/r05_final3_prof.txt 2>&1 || { echo PROF FAIL; tail gpurun_out/r05_final3_prof.txt; exit 1; }
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r05c --write gpurun_out/pmc_write_r05c --out gpurun_out/r05c_pmc_traffic.json || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r05c/wide_kernel_stats.csv 7 24 > gpurun_out/r05_final3_stats.txt || exit 1
head -14 gpurun_out/r05_final3_stats.txt | cut -c1-160
