# Round 5: DDP diagnostic with per-rank initial weights; the stream-overlap probe
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for k in cnn config2; do timeout -k 10 200 python tools/ddp_diag.py $k perrank > gpurun_out/r05_f_ddp_$k.log 2>&1; rc=$?; grep -v "amdgpu.ids\|Gloo" gpurun_out/r05_f_ddp_$k.log | grep "False (\|=avg False" | cut -c1-200 | head -20; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 300 python tools/overlap_probe.py > gpurun_out/r05_f_overlap.log 2>&1; rc=$?; cat gpurun_out/r05_f_overlap.log | grep -v amdgpu; exit $rc
