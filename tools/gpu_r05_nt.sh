# the s20 pixel tests with non-temporal GEMM output stores (default build) and without (ntoff)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in default ntoff; do
  if [ $v = ntoff ]; then export BNN_LIB=$R/abv/ntoff/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_s20.py -v -rf --timeout 120 --timeout-method thread > gpurun_out/r05_nt_s20_$v.log 2>&1; rc=$?
  echo "== $v exit $rc"; grep -E "passed|failed" gpurun_out/r05_nt_s20_$v.log | tail -2; grep -E "^FAILED|assert|Error" gpurun_out/r05_nt_s20_$v.log | cut -c1-250 | head -8
  case $rc in 0|1) ;; *) exit $rc;; esac
done
