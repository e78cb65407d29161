# Round 6, call AE: pack tiles loading whole 256-B row runs (PK_COAL=1, HEAD) against the 16-column
# lanes (abv/pk0) -- the pack / BatchNorm parity tests on HEAD, the scaling probe on both, then
# config 3 / BinCNN graph steps interleaved and config-3 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused.py \
  tests/test_gpu_fp6.py tests/test_gpu_s20.py tests/test_gpu_z16.py tests/test_gpu_q6_handoff.py tests/test_gpu_keep_bits.py \
  tests/test_gpu_net_configs.py tests/test_gpu_cnn_parity.py tests/test_gpu_graph.py > gpurun_out/r06_ae_gpu_tests.log 2>&1 || { echo TESTS FAIL; grep -E "FAILED|Error|assert" gpurun_out/r06_ae_gpu_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r06_ae_gpu_tests.log | tail -1
export TMPDIR=/tmp
for lib in head pk0; do
  if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_r06ae_$lib -o ap -- python3 tools/probe_apply_pack_scale.py > gpurun_out/r06_ae_probe_$lib.log 2>&1 || { echo PROBE FAIL; tail -20 gpurun_out/r06_ae_probe_$lib.log; exit 1; }
  echo "== probe $lib"
  LIB=$lib python3 - <<'PY'
import csv, glob, os
f = glob.glob(f"gpurun_out/prof_r06ae_{os.environ['LIB']}/**/ap_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "sign_pack_tile_k" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
shapes = ["4096x768 qt", "4096x768", "4096x1536 qt", "4096x1536", "4096x3072 qt", "4096x3072", "16384x1536 qt", "16384x1536", "1024x1536 qt", "1024x1536"]
for i in range(0, len(rows), 50):
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows[i:i + 50])
    print(f"{shapes[i // 50]:>14}: median {d[len(d) // 2]:.1f} us")
PY
done
unset BNN_LIB
for rep in 1 2 3; do
  for cfg in mlp cnn; do
    for lib in head pk0; do
      if [ $lib = head ]; then unset BNN_LIB; else export BNN_LIB=$R/abv/$lib/libbnn.so; fi
      tag=${cfg}g_${lib}_$rep
      timeout -k 10 300 python bench.py --config $cfg --graph --steps 300 --warmup 10 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r06_ae_$tag.log 2>&1 || { echo BENCH $tag FAIL; tail -5 gpurun_out/r06_ae_$tag.log; exit 1; }
      echo "$tag: $(tail -1 gpurun_out/r06_ae_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
unset BNN_LIB
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06ae_mlpg -o mlpg --output-format csv -- python3 $R/bench.py --config mlp --graph --steps 50 --warmup 5 --no-cpu-baseline --no-gpu-torch --no-dropin --no-kernel-timing > $R/gpurun_out/r06_ae_prof.log 2>&1 || { echo PROF FAIL; exit 1; }
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/prof_r06ae_mlpg -name 'mlpg_kernel_stats.csv' | head -1) 55 40 > $R/gpurun_out/r06_ae_mlpg_stats.txt
grep -E "kernel time|pack" $R/gpurun_out/r06_ae_mlpg_stats.txt | cut -c1-120
