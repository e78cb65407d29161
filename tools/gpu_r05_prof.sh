# rocprofv3 kernel-trace stats of the wide step at HEAD (and the bench line of the same call)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05_prof -o wide --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-dropin > $R/gpurun_out/r05_prof_bench.log 2>&1; rc=$?
echo "PROF exit $rc"; tail -1 $R/gpurun_out/r05_prof_bench.log | cut -c1-200
find $R/gpurun_out/r05_prof -name "*kernel_stats.csv" | head -3
