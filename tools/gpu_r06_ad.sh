# Round 6, call AD: apply-pack size scaling probe (tools/probe_apply_pack_scale.py) under
# rocprofv3 kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_r06ad -o ap -- python3 tools/probe_apply_pack_scale.py > gpurun_out/r06_ad_probe.log 2>&1 || { echo PROBE FAIL; tail -20 gpurun_out/r06_ad_probe.log; exit 1; }
cat gpurun_out/r06_ad_probe.log | grep "M="
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_r06ad/**/ap_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "sign_pack_tile_k" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# 10 phases of 50 launches, in the probe's order
for i in range(0, len(rows), 50):
    ph = rows[i:i + 50]
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in ph)
    print(f"phase {i // 50}: {ph[0]['Kernel_Name'][:60]} grid {ph[0].get('Grid_Size', ph[0].get('Grid_Size_X', '?'))} median {d[len(d) // 2]:.1f} us min {d[0]:.1f}")
PY
