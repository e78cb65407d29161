# Round-3: BatchNorm-backward statistics in the FP6 dX GEMM epilogue: every -m gpu test, the wide
# bench line, A (BNN_BN_EPI=0) / B wide kernel stats, the MLP graph line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/be_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|^FAILED|^E  " gpurun_out/be_tests.log | cut -c1-300 | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-torch > gpurun_out/be_wide.log 2>&1 || { tail -5 gpurun_out/be_wide.log; exit 1; }
tail -1 gpurun_out/be_wide.log | cut -c1-200
BNN_BN_EPI=0 AB_TOP=12 bash tools/gpu_ab_stats.sh A=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
AB_TOP=12 bash tools/gpu_ab_stats.sh B=distributed-mnist-bnns_amd/lib/libbnn.so || exit 1
timeout -k 10 300 python bench.py --config mlp --graph --steps 200 --warmup 10 --no-cpu-baseline --no-gpu-torch > gpurun_out/be_mlp_g.log 2>&1 || { tail -5 gpurun_out/be_mlp_g.log; exit 1; }
tail -1 gpurun_out/be_mlp_g.log | cut -c1-200
