"""N>1 data-parallel path on CPU: world_size-2 gloo process group (the GPU box runs the same
code over RCCL).  Checks GradExchange against torch's DistributedDataParallel -- the component
the reference wraps around its model (mnist-dist2.py:93) -- and the sampler sharding rule."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT, load_golden


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
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd.parallel import GradExchange
        from oracle.bnn_torch import RefMLP, synthetic_batch

        def make():
            torch.manual_seed(100 + rank)            # different init per rank on purpose
            m = RefMLP(48, 32, 24, p_drop=0.0)
            return m

        ours, ref = make(), make()
        # tiny buckets so the 14 parameters spread over several buckets
        ex = GradExchange(ours, bucket_mb=0.004)
        ddp = torch.nn.parallel.DistributedDataParallel(ref)
        x, t = synthetic_batch(16, 1234 + rank)
        results = {}
        for step in range(2):
            ex.zero_grad()
            ref.zero_grad()
            torch.nn.functional.cross_entropy(ours(x.clone()), t).backward()
            ex.finish()
            torch.nn.functional.cross_entropy(ddp(x.clone()), t).backward()
            for (n, p), q_ in zip(ours.named_parameters(), ref.parameters()):
                assert torch.allclose(p.grad, q_.grad, rtol=1e-5, atol=1e-7), (step, n)
            with torch.no_grad():
                for p, q_ in zip(ours.parameters(), ref.parameters()):
                    p.add_(p.grad, alpha=-0.01)
                    q_.add_(q_.grad, alpha=-0.01)
        results["params"] = [p.detach().clone() for p in ours.parameters()]
        # buffers follow DDP broadcast_buffers semantics: rank 0's stats before each forward,
        # then this rank's own batch update
        for a, b in zip(ours.buffers(), ref.buffers()):
            assert torch.allclose(a.float(), b.float(), rtol=1e-5, atol=1e-6)
        results["nbuckets"] = len(ex.buckets)
        q.put((rank, {k: (v if not isinstance(v, list) else [t.numpy() for t in v])
                      if not torch.is_tensor(v) else v.numpy() for k, v in results.items()}))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def test_gradexchange_matches_torch_ddp_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(out[r], str), out[r]
    assert out[0]["nbuckets"] > 1
    # replicas stay identical: init broadcast + averaged gradients
    for a, b in zip(out[0]["params"], out[1]["params"]):
        np.testing.assert_array_equal(a, b)


def _worker_chunks(rank, world, port, q):
    """The build's own network (bnn_amd.nets.MLP; constructed on CPU, its forward needs libbnn)
    under GradExchange with a bucket cap far below its largest gradients: chunked buckets,
    gradients averaged exactly, coalesced buffer broadcast."""
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd import nets
        from bnn_amd.parallel import GradExchange
        torch.manual_seed(100 + rank)
        model = nets.MLP(48, 32, 24, p_drop=0.0, org_protocol=False, mutate_input=False)
        ex = GradExchange(model, bucket_mb=0.002)        # 524 floats: fc1.weight -> 72 slices
        out = {"nbuckets": len(ex.buckets)}
        sizes = [b.end - b.start for b in ex.buckets]
        out["max_bucket"] = max(sizes)
        out["fc1_slices"] = len(ex._param_buckets[model.fc1.weight])
        params = list(model.parameters())
        out["launch_logs"] = []
        for step in range(2):
            ex.zero_grad()
            coefs = []
            for r in range(world):
                g = torch.Generator().manual_seed(1000 * step + 10 * r)
                coefs.append([torch.randn(p.shape, generator=g) for p in params])
            loss = sum((p * c).sum() for p, c in zip(params, coefs[rank]))
            loss.backward()
            ex.finish()
            out["launch_logs"].append(list(ex.launch_log))
            for i, p in enumerate(params):
                want = sum(coefs[r][i] for r in range(world)) / world
                assert torch.allclose(p.grad, want, rtol=1e-6, atol=1e-7), (step, i)
        # one staging buffer (one broadcast) carries every running stat of every dtype
        assert len(ex._flat_buffers) == 1
        with torch.no_grad():
            model.bn2.running_mean.fill_(float(rank + 1))
            model.bn3.num_batches_tracked.fill_(7 + rank)
        ex.sync_buffers()
        assert torch.all(model.bn2.running_mean == 1.0) and int(model.bn3.num_batches_tracked) == 7
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def test_gradexchange_chunked_buckets_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_chunks, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(out[r], str), out[r]
    assert out[0]["max_bucket"] * 4 <= 0.002 * 2 ** 20
    assert out[0]["fc1_slices"] == 72
    assert out[0]["nbuckets"] > 72
    # RCCL pairs the i-th collective of every rank: both ranks launch the same buckets (same
    # slices) in the same order, every bucket once per step, in bucket order
    assert out[0]["launch_logs"] == out[1]["launch_logs"]
    for log in out[0]["launch_logs"]:
        assert [b for b, _, _ in log] == list(range(out[0]["nbuckets"]))


def test_shard_indices_match_distributed_sampler_golden():
    from bnn_amd.data import shard_indices
    g = load_golden("sampler")
    for key, want in g.items():
        n, ws, r = (int(s[1:] if s[0] == "n" else s[2:] if s.startswith("ws") else s[1:])
                    for s in key.split("_"))
        got = np.array(shard_indices(n, ws, r), np.int64)
        if n >= 1000:
            got = got[:64]
        np.testing.assert_array_equal(got, want)


def _worker_direct_write_count(rank, world, port, q):
    """A weight whose gradient a layer writes straight into its bucket view (direct_write): torch
    still runs that weight's post-accumulate hook (nothing accumulated), and the bucket must not be
    counted complete until every OTHER parameter in it has its gradient -- here the bias used
    before the layer in forward, i.e. after it in backward."""
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd.parallel import GradExchange

        class Net(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.b = torch.nn.Parameter(torch.randn(8))
                self.w = torch.nn.Parameter(torch.randn(4, 8))

        ex_box = []

        class Written(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x, w):
                ctx.save_for_backward(x, w)
                ctx.w = w
                return x @ w.t()

            @staticmethod
            def backward(ctx, g):
                x, w = ctx.saved_tensors
                ex = ex_box[0]
                sink = ex.grad_sink(ctx.w)
                assert sink is not None
                sink.copy_(g.t() @ x)
                ex.grad_written(ctx.w)
                return g @ w, None

        torch.manual_seed(3)
        net = Net()
        seen = []
        # registered before the exchange's own hooks, so it runs first: the bucket holding b must
        # not have been launched yet when b's gradient has just been accumulated
        net.b.register_post_accumulate_grad_hook(lambda p: seen.append(len(ex_box[0].launch_log)))
        ex = GradExchange(net, bucket_mb=1.0, force_collectives=True)
        ex_box.append(ex)
        assert len(ex.buckets) == 1
        x = torch.randn(5, 8)
        for step in range(2):
            ex.zero_grad()
            Written.apply(x + net.b, net.w).square().sum().backward()
            ex.finish()
            g = 2 * ((x + net.b.detach()) @ net.w.detach().t())
            assert torch.allclose(net.w.grad, g.t() @ (x + net.b.detach()), rtol=1e-5, atol=1e-6), step
            assert torch.allclose(net.b.grad, (g @ net.w.detach()).sum(0), rtol=1e-5, atol=1e-6), step
        q.put((rank, {"seen": seen, "writes": ex.direct_writes}))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def test_gradexchange_counts_direct_written_weight_once():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    p = ctx.Process(target=_worker_direct_write_count, args=(0, 1, port, q))
    p.start()
    rank, out = q.get(timeout=120)
    p.join(timeout=60)
    assert not isinstance(out, str), out
    assert out["writes"] == 2
    assert out["seen"] == [0, 0]          # the bucket was launched only after b's gradient
