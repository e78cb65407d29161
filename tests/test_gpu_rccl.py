"""The RCCL branch of the gradient exchange, executed on the one GPU of the test box.

``GradExchange(force_collectives=True)`` over a one-rank ``nccl`` (= RCCL on ROCm) process group,
bound to the device (``device_id``, as bench.py / the trainer do), issues exactly the collectives
an N-GPU run issues: one ``all_reduce(ReduceOp.AVG)`` per bucket slice from the post-accumulate
hooks (and the direct bucket writes) while backward is still running, and the coalesced
per-forward BatchNorm buffer broadcast (DDP broadcast_buffers; replaces mnist-dist2.py:93, the
all-reduce firing inside loss.backward() at :130).  An average over one rank is the identity, so
the training run must be bit-identical to the same run without any exchange: gradients, latent
weights after the fused update, running statistics.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(port, q):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from bnn_amd.parallel import init_rccl
        init_rccl(dev, 0, 1)                      # as bench.py / the trainer: high-priority RCCL stream
        from bnn_amd import nets
        from bnn_amd.data import synthetic_mnist
        from bnn_amd.optim import LatentAdam
        from bnn_amd.parallel import GradExchange

        def make():
            torch.manual_seed(7)
            m = nets.MLP(1024, 512, 512, p_drop=0.3, org_protocol=False, mutate_input=False, fused_bn=True)
            return m.to(dev).train()

        runs = []
        for exchange in (False, True):
            model = make()
            ex = GradExchange(model, bucket_mb=0.5, force_collectives=True) if exchange else None
            opt = LatentAdam(model.parameters(), lr=0.01, clamp_params=nets.binary_params(model))
            torch.manual_seed(99)                      # same dropout seeds in both runs
            rec = []
            for s in range(3):
                x, y = synthetic_mnist(1024, seed=500 + s, device=dev)
                if ex is not None:
                    ex.zero_grad()
                else:
                    for p in model.parameters():
                        p.grad = None
                loss = torch.nn.functional.cross_entropy(model(x), y)
                loss.backward()
                if ex is not None:
                    ex.finish()
                rec.append([p.grad.detach().cpu().numpy().copy() for p in model.parameters()])
                opt.step()
            rec.append([p.detach().cpu().numpy() for p in model.parameters()])
            rec.append([b.detach().cpu().numpy() for b in model.buffers()])
            info = None
            if ex is not None:
                info = {"collectives": ex.collectives, "buckets": len(ex.buckets), "direct": ex.direct_writes}
            runs.append((rec, info))
        dist.destroy_process_group()
        (a, _), (b, info) = runs
        same = all(np.array_equal(x, y) for ra, rb in zip(a, b) for x, y in zip(ra, rb))
        q.put({"same": same, **info})
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put({"error": repr(e), "tb": traceback.format_exc()})


def test_rccl_exchange_one_rank_bit_identical():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        r = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert "error" not in r, r.get("tb", r)
    assert r["same"]
    # every bucket all-reduced on each of the 3 steps, plus one buffer broadcast per forward (and the
    # one at construction); the fused layers wrote fc2's / fc3's weight gradients into their views
    assert r["collectives"] == 3 * r["buckets"] + 3 + 1, r
    assert r["direct"] >= 2, r
