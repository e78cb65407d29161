# Round-5 final artifacts, fourth pass (HEAD after the q6 prefetch guard and the quantiser XCD remap):
# the default bench line, BinCNN / MLP lines (eager + HIP graph), the
# BinCNN through the exchange (eager and graph-captured), rocprofv3 kernel-trace stats of the wide step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r05_final4_bench.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r05_final4_bench.log; exit 1; }
tail -1 gpurun_out/r05_final4_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --config cnn --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final4_cnn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --graph --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final4_cnn_g.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --exchange --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final4_cnn_x.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cnn --graph --exchange --steps 30 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final4_cnn_gx.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch > gpurun_out/r05_final4_mlp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_final4_mlp_g.log 2>&1 || exit 1
for f in cnn cnn_g cnn_x cnn_gx mlp mlp_g; do echo "$f: $(tail -1 gpurun_out/r05_final4_$f.log | grep -o '"ms_per_step": [0-9.]*')"; done
TAG=r05d bash tools/gpu_profile.sh > gpurun_out/r05_final4_prof.txt 2>&1 || { echo PROF FAIL; tail gpurun_out/r05_final4_prof.txt; exit 1; }
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r05d --write gpurun_out/pmc_write_r05d --out gpurun_out/r05d_pmc_traffic.json || exit 1
python3 tools/prof_summary.py gpurun_out/prof_r05d/wide_kernel_stats.csv 7 24 > gpurun_out/r05_final4_stats.txt || exit 1
head -14 gpurun_out/r05_final4_stats.txt | cut -c1-160
