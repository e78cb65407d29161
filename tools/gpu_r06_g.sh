# Round 6, call G: is the one-rank RCCL MLP result a property of the library or of the box/process?
# The same probe on one box: current library twice (two processes), the call-C library once.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for tag in cur1 c_era cur2; do
  if [ $tag = c_era ]; then export BNN_LIB=$R/abv/c_era/libbnn.so; else unset BNN_LIB; fi
  timeout -k 10 300 python -u tools/det_rccl_probe.py 2 > gpurun_out/r06_g_det_$tag.log 2>&1 || { echo DET $tag FAIL; tail -20 gpurun_out/r06_g_det_$tag.log; exit 1; }
  echo "== $tag"; grep -E "^(eager|exchange|graph)" gpurun_out/r06_g_det_$tag.log
done
