"""The RCCL branch of the gradient exchange, executed on the one GPU of the test box.

``GradExchange(force_collectives=True)`` over a one-rank ``nccl`` (= RCCL on ROCm) process group,
bound to the device (``device_id``, as bench.py / the trainer do), issues exactly the collectives
an N-GPU run issues: one ``all_reduce(ReduceOp.AVG)`` per bucket slice from the post-accumulate
hooks (and the direct bucket writes) while backward is still running, and the coalesced
per-forward BatchNorm buffer broadcast (DDP broadcast_buffers; replaces mnist-dist2.py:93, the
all-reduce firing inside loss.backward() at :130).  An average over one rank is the identity, so
the training run must be bit-identical to the same run without any exchange: gradients, latent
weights after the fused update, running statistics.  Workloads: the fused MLP (dropout 0.3) and
the BinCNN of BASELINE config 4 (its BatchNorm2d buffers broadcast per forward, its conv weights
through AccumulateGrad into the bucket views, one ~29 K-parameter bucket).
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


def _worker(port, q, kind):
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
            if kind == "cnn":
                m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
            else:
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


@pytest.mark.parametrize("kind", ["mlp", "cnn"])
def test_rccl_exchange_one_rank_bit_identical(kind):
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q, kind))
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
    if kind == "mlp":
        assert r["direct"] >= 2, r


def _graph_worker(port, q, kind):
    """GraphedStep over a step that contains the exchange: the bucket all-reduces and the buffer
    broadcast captured in the HIP graph with the kernels (RCCL collectives are capturable)."""
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
        init_rccl(dev, 0, 1)
        from bnn_amd import functional as BF
        from bnn_amd import nets
        from bnn_amd.data import synthetic_mnist
        from bnn_amd.graph import GraphedStep
        from bnn_amd.optim import LatentAdam
        from bnn_amd.parallel import GradExchange
        x, y = synthetic_mnist(2048 if kind == "cnn" else 1024, seed=321, device=dev)
        crit = torch.nn.CrossEntropyLoss()
        runs = []
        for graphed in (False, True):
            torch.manual_seed(7)
            if kind == "cnn":
                m = nets.BinCNN(org_protocol=False, mutate_input=False, fused_bn=True)
            else:
                m = nets.MLP(1024, 512, 512, p_drop=0.3, org_protocol=False, mutate_input=False, fused_bn=True)
            m = m.to(dev).train()
            torch.manual_seed(99)                       # the DeviceStep's base dropout seed
            ds = BF.DeviceStep(dev).activate()
            try:
                ex = GradExchange(m, bucket_mb=0.5, force_collectives=True)
                opt = LatentAdam(m.parameters(), lr=0.01, clamp_params=nets.binary_params(m), device_step=ds)

                def step():
                    ex.zero_grad()
                    loss = crit(m(x), y)
                    loss.backward()
                    ex.finish()
                    opt.step()
                    return loss
                losses = []
                if graphed:
                    c0 = ex.collectives
                    g = GraphedStep(step, opt, ds, warmup=2)
                    per_step = (ex.collectives - c0) // 3         # 2 warm-up steps + the capture
                    for _ in range(3):
                        losses.append(float(g().item()))
                else:
                    for i in range(5):
                        loss = step()
                        if i >= 2:
                            losses.append(float(loss.item()))
                    per_step = None
                torch.cuda.synchronize()
                state = [v.detach().cpu().numpy().copy() for v in m.state_dict().values()]
                runs.append((state, losses, per_step, len(ex.buckets)))
                ex.remove()
            finally:
                ds.deactivate()
        dist.destroy_process_group()
        (a, la, _, _), (b, lb, per_step, nb) = runs
        same = all(np.array_equal(u, v) for u, v in zip(a, b))
        q.put({"same": same, "losses": (la, lb), "per_step": per_step, "buckets": nb})
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put({"error": repr(e), "tb": traceback.format_exc()})


@pytest.mark.parametrize("kind", ["mlp", "cnn"])
def test_rccl_exchange_captured_in_graph(kind):
    """The exchange inside GraphedStep (bench.py --graph --exchange; configs 3 and 4 at N > 1 are
    launch-bound): 3 replays of a captured step that issues every bucket all-reduce and the buffer
    broadcast on a one-rank RCCL group equal 3 eager device-step steps with the same exchange, bit
    for bit (parameters, BatchNorm buffers, losses)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_graph_worker, args=(_free_port(), q, kind))
    p.start()
    try:
        r = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert "error" not in r, r.get("tb", r)
    assert r["per_step"] == r["buckets"] + 1, r           # every collective of the step was captured
    assert r["losses"][0] == r["losses"][1], r["losses"]
    assert r["same"]
