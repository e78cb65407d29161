# FP6 GEMM raster-group experiment: build libbnn with BNN_FP6_GROUP=G into a scratch copy, time dX/dW
# shapes and take a FETCH_SIZE pass.  bash tools/gpu_fp6_group.sh "4 8 16"
set -o pipefail
R=$GRAFT_REPO_ROOT
for G in $1; do
  mkdir -p /tmp/g$G && cp -r $R/distributed-mnist-bnns_amd /tmp/g$G/ && cp -r $R/include /tmp/g$G/ && \
  make -s -C /tmp/g$G/distributed-mnist-bnns_amd/csrc -j16 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fvisibility=hidden -DBNN_FP6_GROUP=$G" > /dev/null 2>&1 || { echo "build G=$G failed"; exit 1; }
  export BNN_LIB=/tmp/g$G/distributed-mnist-bnns_amd/lib/libbnn.so
  timeout -k 10 120 python3 $R/tools/gemm_one.py fp6 7 65536 8192 8192 5 || exit 1
  timeout -k 10 120 python3 $R/tools/gemm_one.py fp6 7 8192 8192 65536 5 || exit 1
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/grp$G -o f --output-format csv -- python3 $R/tools/gemm_one.py fp6 7 65536 8192 8192 2 > /dev/null 2>&1 || { echo "pmc G=$G failed"; exit 1; }
  python3 - $R/gpurun_out/grp$G <<'PY'
import csv, glob, sys
rows=[r for f in glob.glob(sys.argv[1]+'/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f)) if 'gemm_fp6' in r['Kernel_Name']]
v=[float(r['Counter_Value']) for r in rows]
print(f"  FETCH dX per launch: {2*1024*sum(v)/len(v)/1e9:.2f} GB over {len(v)} launches")
PY
done
