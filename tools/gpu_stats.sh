# rocprofv3 kernel-trace stats of the default bench step (no PMC): bash tools/gpu_stats.sh TAG [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-stats}; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
python3 $R/tools/prof_summary.py $R/gpurun_out/prof_$TAG/run_kernel_stats.csv 7 30
