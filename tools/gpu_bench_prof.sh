set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o wide --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo PROF FAIL; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -name "*stats*"
