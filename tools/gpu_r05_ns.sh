# how long the FP6 GEMM's epilogue stores take: the wide step with them skipped (timing-only build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in default nostore6 default nostore6; do
  if [ $v = nostore6 ]; then export BNN_LIB=$R/abv/$v/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_ns_wide_$v.log 2>&1; rc=$?
  echo "== $v wide exit $rc"; python3 - "$R/gpurun_out/r05_ns_wide_$v.log" <<'PY'
import json,sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d=json.loads(line); print("ms_per_step", d["ms_per_step"])
        for k,v in sorted(d["kernels"].items(), key=lambda x:-x[1]["share_of_step"])[:3]: print("   %-50s %8.1f us x %.0f"%(k[:50], v["avg_us"], v["launches_per_step"]))
PY
  case $rc in 0|1) ;; *) exit $rc;; esac
done
