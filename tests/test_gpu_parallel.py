"""Data-parallel training on the GPU through GradExchange (libbnn layers, the fused BatchNorm passes,
direct bucket writes) against torch's DistributedDataParallel wrapping an identical copy -- the
component the reference wraps around its model (mnist-dist2.py:93, mnist-dist.py:56,66).  Two ranks
share the one GPU of the test box over gloo (RCCL refuses two ranks on one device; the 8-GPU RCCL
run is the driver's scaling bench).  Workloads:

* ``config2`` -- BASELINE config 2 at its real size: the reference's Net (mnist-dist2.py:46-76,
  infl_ratio 3: 784-3072-1536-768-10, Dropout 0.3) at batch 100 per rank, world size 2, u8 pixels;
* ``mlp`` -- a 512-256-256 MLP at batch 512 with small (0.25 MB) buckets, so the 512 x 512 weights
  span several bucket slices;
* ``cnn`` -- BASELINE config 4's data-parallel form: the BinCNN (conv5x5 1->16 -> BN2d -> Hardtanh ->
  MaxPool, conv5x5 16->32 -> ..., Linear(1568, 10)) on fp32 images, batch 256 per rank.

Bars: gradients of every parameter equal, bit for bit at every step, both DDP's and the exact
average of the ranks' own gradients (a third copy per rank without any exchange, all-gathered; gloo
sums, and a/2 + b/2 and (a + b)/2 round identically); replicas stay identical across ranks (init broadcast + averaged
gradients); BatchNorm buffers follow DDP's broadcast_buffers (rank 0's statistics before each
forward).  Dropout masks differ per rank, as the reference's do, and are the same for both copies
on a rank (the seed drawn from torch's generator, reseeded before each forward).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


WORKLOADS = {
    # kind: (batch per rank, bucket MB, steps)
    "config2": (100, 25.0, 3),
    "mlp": (512, 0.25, 2),
    "cnn": (256, 1.0, 3),
}


def _worker(rank, world, port, q, kind):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd import functional as BF
        from bnn_amd import nets
        from bnn_amd.parallel import GradExchange
        batch, bucket_mb, steps = WORKLOADS[kind]

        def make():
            torch.manual_seed(100 + rank)               # different init per rank on purpose
            if kind == "cnn":
                m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
            elif kind == "config2":
                m = nets.Net(org_protocol=False, mutate_input=False, fused_bn=True)     # p_drop 0.3
            else:
                m = nets.MLP(512, 256, 256, p_drop=0.0, org_protocol=False, mutate_input=False, fused_bn=True)
            return m.cuda().train()

        ours, ref, plain = make(), make(), make()
        ex = GradExchange(ours, bucket_mb=bucket_mb)
        ddp = torch.nn.parallel.DistributedDataParallel(ref, device_ids=[0])
        for p in plain.parameters():              # rank 0's weights, as the exchange / DDP broadcast them
            dist.broadcast(p.data, src=0)
            BF.invalidate_packed(p)
        g = torch.Generator(device="cuda").manual_seed(1234 + rank)
        crit = torch.nn.CrossEntropyLoss()
        written = 0
        for step in range(steps):
            u = torch.randint(0, 256, (batch, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
            u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
            x = u.float().div(255.0) if kind == "cnn" else u
            y = torch.randint(0, 10, (batch,), generator=g, device="cuda")
            ex.zero_grad()
            ref.zero_grad(set_to_none=True)
            for p in plain.parameters():
                p.grad = None
            torch.manual_seed(1000 + 10 * step + rank)      # this rank's dropout seed, for every copy
            crit(ours(x), y).backward()
            written += ex.direct_writes
            ex.finish()
            torch.manual_seed(1000 + 10 * step + rank)
            crit(ddp(x), y).backward()
            torch.manual_seed(1000 + 10 * step + rank)
            crit(plain(x), y).backward()
            for (n, p), q_, r_ in zip(ours.named_parameters(), ref.parameters(), plain.parameters()):
                gs = [torch.empty_like(r_.grad) for _ in range(world)]
                dist.all_gather(gs, r_.grad.contiguous())
                avg = sum(gs) / world                       # the exact average of the ranks' gradients
                assert torch.equal(p.grad, avg), (step, n, "exchange", float((p.grad - avg).abs().max()))
                assert torch.equal(q_.grad, avg), (step, n, "ddp", float((q_.grad - avg).abs().max()))
                r_.grad = avg                               # the plain copy follows the same trajectory
            with torch.no_grad():
                for m_ in (ours, ref, plain):
                    for p in m_.parameters():
                        p.add_(p.grad, alpha=-0.01)
                        BF.invalidate_packed(p)             # raw in-place updates
        for a, b, c in zip(ours.buffers(), ref.buffers(), plain.buffers()):
            assert torch.equal(a, b)
        counters = {"ZQ_HANDOFFS": BF.ZQ_HANDOFFS, "HEAD_CALLS": BF.HEAD_CALLS, "Q6_HANDOFFS": BF.Q6_HANDOFFS}
        out = {"params": [p.detach().cpu().numpy() for p in ours.parameters()], "written": written,
               "nbuckets": len(ex.buckets), "counters": counters}
        ex.remove()
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


@pytest.mark.parametrize("kind", ["config2", "mlp", "cnn"])
def test_gradexchange_matches_ddp_two_ranks_on_gpu(kind):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, kind)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=100) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert not isinstance(out[r], str), out[r]
    if kind == "mlp":
        assert out[0]["nbuckets"] > 3 and out[0]["written"] > 0
    if kind == "config2":
        assert out[0]["written"] > 0 and out[0]["counters"]["HEAD_CALLS"] > 0     # the fused MLP path ran
    if kind == "cnn":
        assert out[0]["counters"]["ZQ_HANDOFFS"] > 0                             # the fused BinCNN path ran
    for a, b in zip(out[0]["params"], out[1]["params"]):
        np.testing.assert_array_equal(a, b)
