# (1) config 2 exchange with hook/launch order; (2) non-temporal GEMM output stores: wide-step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 200 python -u tools/ddp_config2_diag.py 3 > gpurun_out/r05_y_c2.log 2>&1; rc=$?
echo "C2 exit $rc"; grep -v amdgpu gpurun_out/r05_y_c2.log | grep -v "^\[" | grep -v "hand-offs" | cut -c1-1200; ok $rc
for v in default nt default nt; do
  if [ $v = nt ]; then export BNN_LIB=$R/abv/nt/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_z_wide_$v.log 2>&1; rc=$?
  echo "== $v wide exit $rc"; python3 - "$R/gpurun_out/r05_z_wide_$v.log" <<'PY'
import json,sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d=json.loads(line); print("ms_per_step", d["ms_per_step"])
        kt=d.get("kernel_timing",{})
        for k,v in sorted(kt.items(), key=lambda x:-x[1]["share_of_step"])[:9]: print("   %-60s %8.1f us x %.0f"%(k[:60], v["avg_us"], v["launches_per_step"]))
PY
  ok $rc
done
