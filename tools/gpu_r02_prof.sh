# Round-2 profile set: kernel-trace stats + FETCH/WRITE passes of the wide bench step, PMC passes
# over the CNN step (conv kernels), and the MFMA issue-rate probe.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/probes/probe_mfma_rate > $R/gpurun_out/probe_mfma_rate.log 2>&1 || { echo PROBE FAIL; exit 1; }
cat $R/gpurun_out/probe_mfma_rate.log
TAG=r02b bash $R/tools/gpu_profile.sh || exit 1
python3 $R/tools/pmc_summary.py --fetch $R/gpurun_out/pmc_fetch_r02b --write $R/gpurun_out/pmc_write_r02b \
    --out $R/gpurun_out/r02b_pmc_traffic.json || exit 1
BENCH_ARGS="--config cnn" bash $R/tools/gpu_pmc_bench.sh cnn conv || exit 1
