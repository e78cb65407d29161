# Round 5: the FP6 residual plane (dX operands) -- kernel-level tests, the hand-off / z16 bit-identity
# tests, the new CE / conv / guard tests, the config-5 parity + calibration test, then the wide bench
# with and without the residual plane (BNN_FP6_RES=0) on the same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp6.py tests/test_gpu_q6_handoff.py tests/test_gpu_z16.py tests/test_gpu_loss.py tests/test_gpu_s20.py "tests/test_gpu_parity.py::test_conv1_filter_switch_between_forward_and_backward" -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_b_tests.log 2>&1
rc=$?; echo "TESTS exit $rc"; tail -15 gpurun_out/r05_b_tests.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -v -s --timeout 380 --timeout-method thread > gpurun_out/r05_b_wide.log 2>&1
echo "WIDE exit $?"; grep -E "config 5|Hardtanh|per-row|gradient|weight|bias|update max|Error|assert" gpurun_out/r05_b_wide.log | cut -c1-300 | head -40
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/r05_b_bench_res.log 2>&1 || { echo BENCH FAIL; tail -5 gpurun_out/r05_b_bench_res.log; exit 1; }
BNN_FP6_RES=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/r05_b_bench_nores.log 2>&1 || { echo BENCH2 FAIL; exit 1; }
python - <<'PY'
import json
for t in ("res", "nores"):
    d = json.loads(open(f"gpurun_out/r05_b_bench_{t}.log").read().strip().splitlines()[-1])
    ks = {k: v["avg_us"] for k, v in d["kernels"].items() if "fp6" in k or "q6" in k}
    print(t, d["ms_per_step"], d["value"], d["roofline"]["kernel"], d["roofline"]["frac"], ks)
PY
