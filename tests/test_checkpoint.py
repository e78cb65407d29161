"""Latent-weight checkpoints (bnn_amd.checkpoint) on CPU.

The reference's checkpoint (mnist-distributed-BNNS2.py:152-191) saves ``state_dict()`` only, which
for a binarized layer is ``sign(weight.org)``: these tests pin that the build's format keeps the
latent weight, the BatchNorm buffers and the optimizer state, and that the rank-0 save + barrier +
all-ranks load order works over a world_size-2 gloo group."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _nets():
    from bnn_amd import nets
    return nets


def _emulate_forward(model, seed):
    """What a forward under the .org protocol leaves behind (binarized_modules.py:77-79):
    weight.org = the latent weight, weight.data = its sign.  Plus trained-looking BN buffers."""
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if hasattr(m, "org_protocol"):
            latent = torch.empty_like(m.weight).uniform_(-1, 1, generator=g)
            m.weight.org = latent
            m.weight.data = latent.sign()
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.normal_(generator=g)
            m.running_var.uniform_(0.5, 2, generator=g)
            m.num_batches_tracked.fill_(7)


def test_round_trip_keeps_latent_weights_and_buffers(tmp_path):
    from bnn_amd.checkpoint import load_checkpoint, save_checkpoint
    nets = _nets()
    a = nets.MLP(64, 48, 32)
    _emulate_forward(a, 0)
    opt = torch.optim.Adam(a.parameters(), lr=0.01)
    for p in a.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    path = os.path.join(tmp_path, "ck.pt")
    save_checkpoint(path, a, opt, epoch=3)

    b = nets.MLP(64, 48, 32)
    ob = torch.optim.Adam(b.parameters(), lr=0.01)
    assert load_checkpoint(path, b, ob) == 3
    for k in ("fc1", "fc2", "fc3"):
        wa, wb = getattr(a, k).weight, getattr(b, k).weight
        assert torch.equal(wb.org, wa.org), k                     # latent restored ...
        assert torch.equal(wb.data, wa.org.sign()), k             # ... and its sign exposed
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        assert torch.equal(ba, bb), n
    sa, sb = opt.state_dict()["state"], ob.state_dict()["state"]
    assert sa.keys() == sb.keys()
    for i in sa:
        assert torch.equal(sa[i]["exp_avg"], sb[i]["exp_avg"])
        assert torch.equal(sa[i]["exp_avg_sq"], sb[i]["exp_avg_sq"])


def test_plain_state_dict_would_lose_the_latent_weight(tmp_path):
    """The reference's torch.save(state_dict()) restores sign(latent), not the latent."""
    nets = _nets()
    a = nets.MLP(64, 48, 32)
    _emulate_forward(a, 1)
    sd = a.state_dict()
    assert not torch.equal(sd["fc2.weight"], a.fc2.weight.org)
    from bnn_amd.checkpoint import state_with_latents
    sd2, latent = state_with_latents(a)
    assert torch.equal(sd2["fc2.weight"], a.fc2.weight.org)
    assert latent == ["fc1.weight", "fc2.weight", "fc3.weight"]


def test_parameter_held_latents_round_trip(tmp_path):
    """org_protocol = False (the build's trainer): the Parameter is the latent weight."""
    from bnn_amd.checkpoint import load_checkpoint, save_checkpoint
    nets = _nets()
    torch.manual_seed(2)
    a = nets.MLP(64, 48, 32, org_protocol=False, mutate_input=False)
    path = os.path.join(tmp_path, "ck.pt")
    save_checkpoint(path, a, None, epoch=1)
    b = nets.MLP(64, 48, 32, org_protocol=False, mutate_input=False)
    load_checkpoint(path, b)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(pa, pb), n
        assert not hasattr(pb, "org")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, path, q):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bnn_amd import nets
        from bnn_amd.checkpoint import load_checkpoint, save_checkpoint
        m = nets.MLP(32, 32, 32)
        _emulate_forward(m, 10 + rank)         # ranks differ; rank 0's state must win
        save_checkpoint(path, m, None, epoch=5)
        r = nets.MLP(32, 32, 32)
        ep = load_checkpoint(path, r)
        sums = torch.tensor([float(r.fc2.weight.org.sum()), float(r.bn1.running_var.sum()), float(ep)])
        gathered = [torch.zeros(3) for _ in range(world)]
        dist.all_gather(gathered, sums)
        ref = nets.MLP(32, 32, 32)
        _emulate_forward(ref, 10)
        ok = all(torch.equal(g, gathered[0]) for g in gathered) and \
            float(gathered[0][0]) == float(ref.fc2.weight.org.sum()) and float(gathered[0][2]) == 5.0
        dist.destroy_process_group()
        q.put((rank, ok, ""))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e)))


def test_rank0_save_barrier_load_gloo(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = os.path.join(tmp_path, "dist.pt")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, err in res:
        assert ok, f"rank {rank}: {err}"


@pytest.mark.gpu
def test_trainer_checkpoint_and_resume_on_gpu(tmp_path):
    """bnn_amd.trainer --checkpoint / --resume on one GPU: epoch 1 writes the latent weights and
    Adam state, the resumed run starts at epoch 2 from exactly those tensors."""
    from bnn_amd import trainer
    from bnn_amd.checkpoint import load_checkpoint
    path = os.path.join(tmp_path, "tr.pt")
    common = ["--model", "small", "--max-steps", "3", "--dataset-size", "512", "--batch-size", "128",
              "--log-interval", "100"]
    m1 = trainer.train(0, trainer.parse(common + ["--epochs", "1", "--checkpoint", path]))
    blob = torch.load(path, weights_only=True)
    assert blob["epoch"] == 1
    for k, v in m1.state_dict().items():
        assert torch.equal(blob["model"][k].cuda(), v), k
    m2 = trainer.train(0, trainer.parse(common + ["--epochs", "2", "--resume", path, "--checkpoint", path]))
    assert torch.load(path, weights_only=True)["epoch"] == 2
    fresh = trainer.nets.SmallNet(org_protocol=False, mutate_input=False, fused_bn=True).cuda()
    assert load_checkpoint(path, fresh) == 2
    for (n, pa), pb in zip(m2.named_parameters(), fresh.parameters()):
        assert torch.equal(pa, pb), n
