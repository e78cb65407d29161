# Round 5: config-5 parity + calibration with the residual plane, the wide bench with / without it,
# then the determinism probe and the DDP / RCCL tests (test failures there do not stop the script).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide_step.py::test_wide_step_config5_vs_float64 -v -s --timeout 380 --timeout-method thread > gpurun_out/r05_d_wide.log 2>&1
rc=$?; echo "WIDE exit $rc"; grep -E "config 5|Hardtanh|per-row|gradient|weight|bias|update max|Error|assert" gpurun_out/r05_d_wide.log | cut -c1-300 | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/r05_d_bench_res.log 2>&1 || { echo BENCH FAIL; tail -5 gpurun_out/r05_d_bench_res.log; exit 1; }
BNN_FP6_RES=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/r05_d_bench_nores.log 2>&1 || { echo BENCH2 FAIL; exit 1; }
python - <<'PY'
import json
for t in ("res", "nores"):
    d = json.loads(open(f"gpurun_out/r05_d_bench_{t}.log").read().strip().splitlines()[-1])
    ks = {k: v["avg_us"] for k, v in d["kernels"].items() if "fp6" in k or "q6" in k}
    print(t, d["ms_per_step"], d["value"], d["roofline"]["kernel"], d["roofline"]["frac"], d.get("binary_gemm_tops"), d.get("fc1_tops"), ks)
PY
for k in config2 mlp cnn; do timeout -k 10 120 python tools/det_probe.py $k > gpurun_out/r05_d_det_$k.log 2>&1; rc=$?; cat gpurun_out/r05_d_det_$k.log | tail -3; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_rccl.py -v --timeout 300 --timeout-method thread > gpurun_out/r05_d_dist.log 2>&1
echo "DIST exit $?"; grep -E "PASS|FAIL|Error" gpurun_out/r05_d_dist.log | cut -c1-400 | tail -20
