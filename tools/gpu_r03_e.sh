# Round-3 GPU call E: bench.py --exchange (one-rank RCCL group issuing every bucket all-reduce and
# the buffer broadcast) under a rocprofv3 kernel trace; the collectives' overlap with backward.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --rccl-trace --stats -d $R/gpurun_out/prof_exchange -o exch --output-format csv -- \
  python3 $R/bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-gpu-torch --no-kernel-timing \
  > $R/gpurun_out/bench_exchange.log 2>&1 || { echo "EXCHANGE FAIL"; tail -20 $R/gpurun_out/bench_exchange.log; exit 1; }
tail -1 $R/gpurun_out/bench_exchange.log | cut -c1-400
python3 $R/tools/comm_overlap.py $(find $R/gpurun_out/prof_exchange -name "*kernel_trace.csv" | head -1) \
  $(find $R/gpurun_out/prof_exchange -name "*rccl_api_trace.csv" | head -1) \
  > $R/gpurun_out/comm_overlap.txt && cat $R/gpurun_out/comm_overlap.txt
