"""BASELINE config 2 on the GPU: the build's own fused binarized MLP (libbnn layers, u8 pixels, the
fused BatchNorm passes, direct bucket writes) trained data-parallel by GradExchange, against torch's
DistributedDataParallel wrapping an identical copy -- the component the reference wraps around its
model (mnist-dist2.py:93).  Two ranks share the one GPU of the test box over gloo (RCCL refuses two
ranks on one device; the 8-GPU RCCL run is the driver's scaling bench).

* gradients of every parameter equal DDP's bit for bit at every step (gloo sums; a/2 + b/2 and
  (a + b)/2 round identically);
* replicas stay identical across ranks (init broadcast + averaged gradients);
* BatchNorm buffers follow DDP's broadcast_buffers (rank 0's statistics before each forward).
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


def _worker(rank, world, port, q):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd import nets
        from bnn_amd.parallel import GradExchange

        def make():
            torch.manual_seed(100 + rank)               # different init per rank on purpose
            return nets.MLP(512, 256, 256, p_drop=0.0, org_protocol=False, mutate_input=False,
                            fused_bn=True).cuda().train()

        ours, ref = make(), make()
        ex = GradExchange(ours, bucket_mb=0.25)         # the 512x512 weight spans several buckets
        ddp = torch.nn.parallel.DistributedDataParallel(ref, device_ids=[0])
        g = torch.Generator(device="cuda").manual_seed(1234 + rank)
        u = torch.randint(0, 256, (512, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
        y = torch.randint(0, 10, (512,), generator=g, device="cuda")
        crit = torch.nn.CrossEntropyLoss()
        written = 0
        for step in range(2):
            ex.zero_grad()
            ref.zero_grad(set_to_none=True)
            crit(ours(u), y).backward()
            written += ex.direct_writes
            ex.finish()
            crit(ddp(u), y).backward()
            for (n, p), q_ in zip(ours.named_parameters(), ref.parameters()):
                assert torch.equal(p.grad, q_.grad), (step, n, float((p.grad - q_.grad).abs().max()))
            with torch.no_grad():
                for p, q_ in zip(ours.parameters(), ref.parameters()):
                    p.add_(p.grad, alpha=-0.01)
                    q_.add_(q_.grad, alpha=-0.01)
            from bnn_amd import functional as BF
            for p, q_ in zip(ours.parameters(), ref.parameters()):   # raw in-place updates
                BF.invalidate_packed(p)
                BF.invalidate_packed(q_)
        for a, b in zip(ours.buffers(), ref.buffers()):
            assert torch.equal(a, b)
        out = {"params": [p.detach().cpu().numpy() for p in ours.parameters()], "written": written,
               "nbuckets": len(ex.buckets)}
        ex.remove()
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def test_fused_mlp_gradexchange_matches_ddp_two_ranks_on_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
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
    assert out[0]["nbuckets"] > 3 and out[0]["written"] > 0
    for a, b in zip(out[0]["params"], out[1]["params"]):
        np.testing.assert_array_equal(a, b)
