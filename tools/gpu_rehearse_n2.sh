# Rehearsal of the N > 1 bench path (RCCL process group, GradExchange buckets, buffer broadcast,
# max-over-ranks timing) with 2 ranks sharing the one GPU of a gpurun box, at a reduced batch,
# over gloo (RCCL refuses two ranks on one device).
# Not a scaling measurement: both ranks time-share one device.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BNN_BENCH_ONE_DEVICE=1 BNN_BENCH_BACKEND=${BACKEND:-gloo} timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch ${BATCH:-8192} \
  --no-kernel-timing ${BENCH_ARGS} > gpurun_out/rehearse_n2.log 2>&1
rc=$?
echo "N2 EXIT $rc"; grep -v "^\s*$" gpurun_out/rehearse_n2.log | tail -15 | cut -c1-400
exit $rc
