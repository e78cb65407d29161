# Round-5 final profile of HEAD's wide step (no drop-in / torch comparators in the traced process):
# rocprofv3 kernel-trace stats + FETCH / WRITE PMC passes -> per-kernel traffic
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
rm -rf gpurun_out/prof_r05 gpurun_out/pmc_fetch_r05 gpurun_out/pmc_write_r05
TAG=r05 bash tools/gpu_profile.sh > gpurun_out/r05_final_prof.txt 2>&1 || { echo PROF FAIL; tail gpurun_out/r05_final_prof.txt; exit 1; }
cd $R
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch_r05 --write gpurun_out/pmc_write_r05 --out gpurun_out/r05_pmc_traffic.json || exit 1
python3 tools/prof_summary.py $(find gpurun_out/prof_r05 -name 'wide_kernel_stats.csv' | head -1) 7 24 > gpurun_out/r05_final_stats.txt || exit 1
head -16 gpurun_out/r05_final_stats.txt | cut -c1-160
