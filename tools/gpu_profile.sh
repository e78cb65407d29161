# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench step.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-300
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo PMC1 FAIL; tail -20 $R/gpurun_out/pmc_fetch_$TAG.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o wide --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || { echo PMC2 FAIL; tail -20 $R/gpurun_out/pmc_write_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG $R/gpurun_out/pmc_fetch_$TAG $R/gpurun_out/pmc_write_$TAG -name "*.csv" | head -20
