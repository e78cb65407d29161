# Round 4: the fc3 forward FP4 GEMM (int16 output) at the wide shape -- full / no k loop (the
# epilogue alone) / no stores / full, each library in its own process (tools/fp4_diag.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for lib in distributed-mnist-bnns_amd/lib/libbnn.so ab/nomain/libbnn.so ab/nostore/libbnn.so distributed-mnist-bnns_amd/lib/libbnn.so; do
  BNN_LIB=$R/$lib timeout -k 10 120 python tools/fp4_diag.py >> gpurun_out/r04_fp4_diag.log 2>&1 || { echo FP4DIAG FAIL; tail -5 gpurun_out/r04_fp4_diag.log; exit 1; }
done
grep "per launch" gpurun_out/r04_fp4_diag.log
