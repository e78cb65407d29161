# Round-3 GPU calls D + E in one: q6 tests, A/B/C kernel stats, then the RCCL exchange trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r03_f.sh || exit $?
bash tools/gpu_r03_e.sh
