# FP6 GEMM epilogue stagger A/B (BNN_FP6_STAGGER ticks of 10 ns per phase; 0 = off)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for st in 0 500 1000 2000 0 1000; do
  BNN_FP6_STAGGER=$st timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_st_$st.log 2>&1; rc=$?
  echo "== stagger $st exit $rc"; python3 - "$R/gpurun_out/r05_st_$st.log" <<'PY'
import json,sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d=json.loads(line); print("ms_per_step", d["ms_per_step"])
        for k,v in sorted(d["kernels"].items(), key=lambda x:-x[1]["share_of_step"])[:2]: print("   %-50s %8.1f us x %.0f"%(k[:50], v["avg_us"], v["launches_per_step"]))
PY
  case $rc in 0|1) ;; *) exit $rc;; esac
done
