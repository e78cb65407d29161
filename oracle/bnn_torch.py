"""CPU restatement of the reference's training path in plain torch (fp32) -- TEST / BASELINE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
this module.  It is what the reference runs on a CPU: torch's fp32 ``F.linear`` / ``F.conv2d`` on
sign()ed operands, ``BatchNorm1d``, ``Hardtanh``, ``torch.optim.Adam`` and the ``.org``
protocol.  bench.py times it on the GPU box's host cores as the ``"port"`` CPU baseline
(the reference source itself never travels there): configs 1 (single process) and 2 (gloo
DDP, ``time_training_gloo``), and the bench config itself; run with GPU tensors it is the naive
"reference semantics on torch fp32 GEMMs" comparator.  Pinned to the reference's outputs by
tests/test_oracle_golden.py::test_torch_restatement_* against tests/golden/*.npz.

Restated from: models/binarized_modules.py:11-13 (Binarize), :68-85 (BinarizeLinear),
:87-107 (BinarizeConv2d); mnist-dist2.py:46-76 (Net), :118-137 (train step).
"""
import json
import os
import socket
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as tF


def _latent_sign(p):
    # binarized_modules.py:77-79 -- the latent copy is made once, its sign is exposed in .data
    if not hasattr(p, "org"):
        p.org = p.data.clone()
    p.data = p.org.sign()


class RefLinear(nn.Linear):
    """BinarizeLinear semantics on CPU (binarized_modules.py:73-85)."""

    def forward(self, inp):
        if inp.size(1) != 784:
            inp.data = inp.data.sign()
        _latent_sign(self.weight)
        y = tF.linear(inp, self.weight)
        if self.bias is not None:
            self.bias.org = self.bias.data.clone()
            y += self.bias.view(1, -1).expand_as(y)
        return y


class RefConv2d(nn.Conv2d):
    """BinarizeConv2d semantics on CPU (binarized_modules.py:93-107)."""

    def forward(self, inp):
        if inp.size(1) != 3:
            inp.data = inp.data.sign()
        _latent_sign(self.weight)
        y = tF.conv2d(inp, self.weight, None, self.stride, self.padding, self.dilation, self.groups)
        if self.bias is not None:
            self.bias.org = self.bias.data.clone()
            y += self.bias.view(1, -1, 1, 1).expand_as(y)
        return y


class RefMLP(nn.Module):
    """mnist-dist2.py:46-76 topology with explicit widths."""

    def __init__(self, h1, h2, h3, p_drop=0.3):
        super().__init__()
        self.fc1, self.bn1 = RefLinear(784, h1), nn.BatchNorm1d(h1)
        self.fc2, self.bn2 = RefLinear(h1, h2), nn.BatchNorm1d(h2)
        self.fc3, self.bn3 = RefLinear(h2, h3), nn.BatchNorm1d(h3)
        self.fc4 = nn.Linear(h3, 10)
        self.drop = nn.Dropout(p_drop)

    def forward(self, x):
        x = x.view(-1, 784)
        x = tF.hardtanh(self.bn1(self.fc1(x)))
        x = tF.hardtanh(self.bn2(self.fc2(x)))
        x = tF.hardtanh(self.bn3(self.drop(self.fc3(x))))
        return tF.log_softmax(self.fc4(x), dim=1)


class RefCNN(nn.Module):
    """The build's BinCNN (BASELINE config 4) with the reference's CPU layers: BinarizeConv2d
    (binarized_modules.py:87-107) -> BatchNorm2d -> Hardtanh -> MaxPool2d(2), twice, then
    Linear(1568, 10) and LogSoftmax (mnist-dist.py:31-51 ConvNet template)."""

    def __init__(self):
        super().__init__()
        self.c1, self.b1 = RefConv2d(1, 16, 5, padding=2), nn.BatchNorm2d(16)
        self.c2, self.b2 = RefConv2d(16, 32, 5, padding=2), nn.BatchNorm2d(32)
        self.fc = nn.Linear(7 * 7 * 32, 10)

    def forward(self, x):
        x = tF.max_pool2d(tF.hardtanh(self.b1(self.c1(x))), 2, 2)
        x = tF.max_pool2d(tF.hardtanh(self.b2(self.c2(x))), 2, 2)
        return tF.log_softmax(self.fc(x.reshape(x.size(0), -1)), dim=1)


def train_step(model, opt, x, target, org_protocol=True):
    """mnist-dist2.py:122-137 (org protocol) or mnist-dist3.py:113-119 (without)."""
    opt.zero_grad()
    loss = tF.cross_entropy(model(x), target)
    loss.backward()
    params = list(model.parameters())
    if org_protocol:
        for p in params:
            if hasattr(p, "org"):
                p.data.copy_(p.org)
    opt.step()
    if org_protocol:
        for p in params:
            if hasattr(p, "org"):
                p.org.copy_(p.data.clamp_(-1, 1))
    return loss.item()


def synthetic_batch(n, seed, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    u = torch.rand((n, 1, 28, 28), generator=g)
    v = torch.randint(1, 256, (n, 1, 28, 28), generator=g).float()
    x = torch.where(u < 0.807, torch.zeros_like(v), v) / 255.0
    return x.to(device), torch.randint(0, 10, (n,), generator=g).to(device)


def time_training(widths, batch, threads, budget_s=10.0, max_steps=50, min_steps=2, warmup=1, device="cpu"):
    """Time the reference training step (fp32 torch; on `threads` host threads, or on a GPU with
    device="cuda" -- the naive "reference semantics on torch fp32 GEMMs" comparator); widths =
    (h1, h2, h3) for the MLPs or "cnn" for RefCNN.

    Returns (samples_per_s, steps, seconds)."""
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    model = (RefCNN() if widths == "cnn" else RefMLP(*widths)).to(device)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    x, t = synthetic_batch(batch, 1234, device)
    sync = torch.cuda.synchronize if device != "cpu" else (lambda: None)
    for _ in range(warmup):
        train_step(model, opt, x.clone(), t)
    sync()
    steps, t0 = 0, time.perf_counter()
    while steps < max_steps:
        train_step(model, opt, x.clone(), t)
        steps += 1
        el = time.perf_counter() - t0
        if steps >= min_steps and el >= budget_s:
            break
    sync()
    el = time.perf_counter() - t0
    return batch * steps / el, steps, el


# ----------------------------------------------------------------------------- gloo DDP (config 2)
def _gloo_rank(rank, world, port, widths, batch, threads, budget_s, q):
    """One rank of the reference's data-parallel loop: gloo process group, DDP over the CPU
    restatement (mnist-dist2.py:83, :93), per-rank shard of the batch, .org protocol."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(threads)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.parallel.DistributedDataParallel(RefMLP(*widths))
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    x, t = synthetic_batch(batch, 1234 + rank)
    train_step(model, opt, x.clone(), t)
    steps, t0 = 0, time.perf_counter()
    while True:
        train_step(model, opt, x.clone(), t)
        steps += 1
        el = torch.tensor([time.perf_counter() - t0])
        dist.all_reduce(el, op=dist.ReduceOp.MAX)   # every rank agrees when to stop
        if steps >= 2 and float(el) >= budget_s:
            break
    if rank == 0:
        q.put((steps, float(el)))
    dist.destroy_process_group()


def time_training_gloo(widths, batch, world, threads_per_rank, budget_s=8.0):
    """BASELINE config 2: the same MLP step under gloo DDP with `world` CPU ranks on this host
    (threads split per rank).  `batch` is per rank; returns (total samples/s, steps, seconds)."""
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, widths, batch, threads_per_rank, budget_s, q))
             for r in range(world)]
    for p in procs:
        p.start()
    steps, el = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    return batch * world * steps / el, steps, el


if __name__ == "__main__":
    # python -m oracle.bnn_torch gloo H1 H2 H3 BATCH WORLD THREADS BUDGET  -> one JSON line
    if len(sys.argv) == 9 and sys.argv[1] == "gloo":
        h1, h2, h3, b, w, th = (int(v) for v in sys.argv[2:8])
        sps, n, secs = time_training_gloo((h1, h2, h3), b, w, th, float(sys.argv[8]))
        print(json.dumps({"samples_per_s": sps, "steps": n, "seconds": secs}), flush=True)
