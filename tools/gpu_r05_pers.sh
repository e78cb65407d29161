# persistent FP6 GEMM: parity (bit-identical to one workgroup per tile), then the wide step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp6.py -x -v --timeout 200 --timeout-method thread -k "persistent or panel or residual" > gpurun_out/r05_pers_tests.log 2>&1; rc=$?
echo "TESTS exit $rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r05_pers_tests.log | cut -c1-200 | tail -14
[ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  BNN_FP6_PERS=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_pers_wide_$v.log 2>&1; rc=$?
  echo "== persistent=$v exit $rc"; python3 - "$R/gpurun_out/r05_pers_wide_$v.log" <<'PY'
import json,sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d=json.loads(line); print("ms_per_step", d["ms_per_step"])
        for k,v in sorted(d["kernels"].items(), key=lambda x:-x[1]["share_of_step"])[:3]: print("   %-50s %8.1f us x %.0f"%(k[:50], v["avg_us"], v["launches_per_step"]))
PY
  case $rc in 0|1) ;; *) exit $rc;; esac
done
