# Round 5: DDP-vs-GradExchange diagnostic (which side differs from the hand-made average)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for k in cnn config2; do timeout -k 10 200 python tools/ddp_diag.py $k > gpurun_out/r05_e_ddp_$k.log 2>&1; rc=$?; grep -v "amdgpu.ids" gpurun_out/r05_e_ddp_$k.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; done
