# GPU session: variant exactness tests, then the GEMM sweep.  Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "variant" > gpurun_out/parity.log 2>&1 || { echo PARITY FAIL; tail -30 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
timeout -k 10 400 python -u tools/gemm_sweep.py --reps ${REPS:-3} ${SWEEP_ARGS:-} > gpurun_out/sweep.log 2>&1 || { echo SWEEP FAIL; tail -20 gpurun_out/sweep.log; exit 1; }
cut -c1-170 gpurun_out/sweep.log
