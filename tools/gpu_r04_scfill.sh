# Round 4: FP6 scale slabs allocated without a zero fill -- the FP6 / q6 / fused / wide tests,
# then the wide bench with kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp6.py tests/test_gpu_q6_handoff.py tests/test_gpu_fused.py tests/test_gpu_wide_step.py tests/test_gpu_head.py tests/test_gpu_net_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_scfill_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r04_scfill_tests.log; [ $rc = 0 ] || { grep -E "Error|assert" gpurun_out/r04_scfill_tests.log | head; exit 1; }
bash tools/gpu_stats.sh scfill > gpurun_out/r04_scfill_stats.txt 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_scfill.log
grep -E "Fill|kernel time" gpurun_out/r04_scfill_stats.txt | cut -c1-150
