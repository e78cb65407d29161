"""The reference's own data-parallel configuration on the GPU: torch ``DistributedDataParallel``
wrapped around a ``Net`` built from the drop-in ``models.binarized_modules`` (torch BatchNorm1d,
Hardtanh, Dropout, LogSoftmax around it), trained by the reference's loop verbatim.

* ``org``    -- mnist-dist2.py:46-76 (Net, infl_ratio 3: 784-3072-1536-768-10, Dropout 0.3),
  :83,93 (``optim.Adam`` on the model's parameters, then ``nn.parallel.DistributedDataParallel``),
  :122-137 (zero_grad, forward, CrossEntropyLoss, backward, the ``.org`` restore -> ``Adam.step()``
  -> clamp loop); BASELINE config 2: batch 100 per rank, world size 2.
* ``frozen`` -- mnist-dist3.py:38-67 (Net 784-192-192-192-10), :78-84 (Adam, DDP), :113-119 (the
  loop without the ``.org`` protocol: Adam updates the binarised copy that the next forward
  overwrites, so the binary weights stay frozen at their initial signs), batch 64 per rank.
* ``org-bn`` -- ``org`` with the Net's bn1..bn3 swapped for ``bnn_amd.nn.BatchNorm1d`` on the
  drop-in side (the oracle keeps torch's): the BatchNorm outputs within 1e-5 of torch's, then
  anchored like z1 (ties on the batch mean, see the worker), and the same bars.

Inside DDP's forward the drop-in layers reassign ``weight.data = sign(weight.org)``
(binarized_modules.py:77-79) and mutate their input (:76), and DDP's all-reduce fires inside
``loss.backward()`` -- the ways a module replacement could break under DDP.  The comparator is
the same script on the oracle's torch restatement of the modules (``oracle.bnn_torch.RefLinear``:
torch fp32 GEMMs on sign()ed operands, on the same GPU), also under DDP, with the same per-rank
initial weights, batches and dropout masks (torch's generator reseeded before each forward).

Bars (north_star: every gradient within 1e-5 norm-wise; ``conftest.rel_err``):
* Both: the oracle runs from the drop-in's fc1 output z1 (forward-hook anchoring, as every whole-net
  test here): z1 is fp32-rounded differently by any two implementations of fc1 (its input is
  continuous), and pixels in multiples of 1/255 put elements exactly on bn1's batch mean, whose
  sign that rounding decides (test_gpu_net_configs.py: z1 itself is checked against float64 there).
* ``frozen`` runs free for 3 steps (the binary weights cannot diverge): loss and log-probs
  <= 1e-5, every gradient <= 1e-5 (the fc biases feed BatchNorm: their exact gradient is 0 and both
  sides hold rounding noise, checked absolute), the learned BatchNorm and fc4 parameters <= 1e-5.
* ``org`` is anchored per step: before steps 1 and 2 the oracle copy takes the drop-in's state
  (latent ``.org`` weights, biases, BatchNorm buffers, Adam moments), so each step is compared from
  one state -- free-running, the first Adam step moves a latent by ~lr * sign(g) and any element
  whose gradient is within rounding of 0 can step the other way and flip its sign at the next
  forward ("Why forcing").  Per step: loss and log-probs <= 1e-5, every gradient
  <= 1e-5; after the update, every latent ``.org`` equal to float64 Adam + clamp from its pre-step
  value and moments on the all-reduced gradient within 1e-6 (the restore -> step -> clamp loop
  worked under DDP); the latents where the oracle's own update differs by > 1e-6 are counted and
  printed (Adam's lr * g / (|g| + eps) turns a rounding-level gradient difference into a different
  step wherever |g| is within a few orders of eps = 1e-8, e.g. fc1 columns of faint pixels).
Also asserted: DDP kept the two ranks' replicas identical (init broadcast + averaged gradients).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

TOL = 1e-5
FC_BIAS = ("fc1.bias", "fc2.bias", "fc3.bias")
BINARY_W = ("fc1.weight", "fc2.weight", "fc3.weight")
CASES = {
    # kind: (widths, batch per rank, org protocol, drop-in BatchNorm1d on our side)
    "org": ((3072, 1536, 768), 100, True, False),        # mnist-dist2.py
    "frozen": ((192, 192, 192), 64, False, False),       # mnist-dist3.py
    "org-bn": ((3072, 1536, 768), 100, True, True),      # mnist-dist2.py + bnn_amd.nn.BatchNorm1d
}
STEPS = 3
LR = 0.01


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _make_net(linear, widths, bn=nn.BatchNorm1d):
    """mnist-dist2.py:46-76 / mnist-dist3.py:38-67 with the Linear (and BatchNorm1d) class injected."""
    h1, h2, h3 = widths

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1 = linear(784, h1)
            self.htanh1 = nn.Hardtanh()
            self.bn1 = bn(h1)
            self.fc2 = linear(h1, h2)
            self.htanh2 = nn.Hardtanh()
            self.bn2 = bn(h2)
            self.fc3 = linear(h2, h3)
            self.htanh3 = nn.Hardtanh()
            self.bn3 = bn(h3)
            self.fc4 = nn.Linear(h3, 10)
            self.logsoftmax = nn.LogSoftmax(dim=1)
            self.drop = nn.Dropout(0.3)

        def forward(self, x):
            x = x.view(-1, 28 * 28)
            x = self.htanh1(self.bn1(self.fc1(x)))
            x = self.htanh2(self.bn2(self.fc2(x)))
            x = self.fc3(x)
            x = self.drop(x)
            x = self.htanh3(self.bn3(x))
            return self.logsoftmax(self.fc4(x))

    return Net()


def _reference_step(model, optimizer, criterion, data, target, org_protocol):
    """mnist-dist2.py:122-137 (org_protocol) / mnist-dist3.py:113-119, verbatim in behaviour; the
    gradients are snapshotted after DDP's all-reduce (inside backward) and before the update."""
    optimizer.zero_grad()
    output = model(data)
    loss = criterion(output, target)
    optimizer.zero_grad()
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.module.named_parameters()}
    pre = {}                                  # latent + Adam state before the update (the update check)
    for n, p in model.module.named_parameters():
        st = optimizer.state.get(p, {})
        pre[n] = (p.org.detach().clone() if hasattr(p, "org") else None,
                  {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()})
    if org_protocol:
        for p in list(model.parameters()):
            if hasattr(p, "org"):
                p.data.copy_(p.org)
    optimizer.step()
    if org_protocol:
        for p in list(model.parameters()):
            if hasattr(p, "org"):
                p.org.copy_(p.data.clamp_(-1, 1))
    return loss.detach(), output.detach(), grads, pre


def _anchor(dst_model, dst_opt, src_model, src_opt):
    """The oracle copy takes the drop-in copy's whole training state."""
    with torch.no_grad():
        for (n, d), s in zip(dst_model.module.named_parameters(), src_model.module.parameters()):
            d.data.copy_(s.data)
            if hasattr(s, "org"):
                d.org = s.org.detach().clone()
        for d, s in zip(dst_model.module.buffers(), src_model.module.buffers()):
            d.copy_(s)
        for d, s in zip(dst_model.module.parameters(), src_model.module.parameters()):
            st = src_opt.state.get(s)
            if st:
                dst_opt.state[d] = {k: v.detach().clone() for k, v in st.items()}


def _rel(a, b):
    a, b = a.double(), b.double()
    nb = float(b.norm())
    return float((a - b).norm()) / (nb if nb > 0 else 1.0)


def _worker(rank, world, port, q, kind):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from models.binarized_modules import BinarizeLinear
        from oracle.bnn_torch import RefLinear
        widths, batch, org, dropin_bn = CASES[kind]
        from bnn_amd.nn import BatchNorm1d

        def build(linear, bn=nn.BatchNorm1d):
            torch.manual_seed(100 + rank)          # per-rank init, as mnist-dist2.py: DDP broadcasts rank 0's
            m = _make_net(linear, widths, bn).cuda().train()
            opt = torch.optim.Adam(m.parameters(), lr=LR)                       # mnist-dist2.py:89
            return nn.parallel.DistributedDataParallel(m, device_ids=[0]), opt  # :93

        ours, opt_o = build(BinarizeLinear, BatchNorm1d if dropin_bn else nn.BatchNorm1d)
        ref, opt_r = build(RefLinear)
        # z1 anchoring: the oracle's fc1 output takes the drop-in's value (its gradient still flows
        # through the oracle's own fc1).  fc1's input is continuous, z1 carries each implementation's
        # fp32 rounding, and an element on bn1's batch mean (pixels are multiples of 1/255, so exact
        # ties occur: ~10 per step at 3072 columns) takes whichever sign that rounding gives it.
        z1 = {}
        ours.module.fc1.register_forward_hook(lambda m, i, o: z1.__setitem__("v", o.detach()))
        ref.module.fc1.register_forward_hook(lambda m, i, o: z1["v"] + (o - o.detach()))   # exactly z1
        bn_out, bn_err = {}, []
        if dropin_bn:
            # the BatchNorm outputs anchored the same way: both sides' outputs are compared (<= 1e-5
            # norm-wise), then the oracle continues from ours.  libbnn's batch mean carries a lo part
            # (x - mean = (x - hi) - lo) where torch's is one fp32 value, so an element on the batch
            # mean (z1 takes discrete values: pixel sums / 255) can come out as +-tiny on one side and
            # exactly 0 on the other, and the next layer's sign() turns that into a different ternary
            # input.  Each side's own BatchNorm backward still runs.
            for name in ("bn1", "bn2", "bn3"):
                getattr(ours.module, name).register_forward_hook(
                    lambda m, i, o, name=name: bn_out.__setitem__(name, o.detach()))

                def take(m, i, o, name=name):
                    bn_err.append(_rel(bn_out[name], o.detach()))
                    return bn_out[name] + (o - o.detach())
                getattr(ref.module, name).register_forward_hook(take)
        crit = nn.CrossEntropyLoss()
        g = torch.Generator(device="cuda").manual_seed(1234 + rank)
        report = []
        for step in range(STEPS):
            u = torch.randint(0, 256, (batch, 1, 28, 28), generator=g, device="cuda").to(torch.uint8)
            u = torch.where(torch.rand(u.shape, generator=g, device="cuda") < 0.807, torch.zeros_like(u), u)
            data = u.float().div(255.0)                       # transforms.ToTensor()
            target = torch.randint(0, 10, (batch,), generator=g, device="cuda")
            if org and step > 0:
                _anchor(ref, opt_r, ours, opt_o)
            torch.manual_seed(1000 + 10 * step + rank)        # this rank's dropout mask, for both copies
            lo, out_o, g_o, pre_o = _reference_step(ours, opt_o, crit, data.clone(), target, org)
            torch.manual_seed(1000 + 10 * step + rank)
            lr_, out_r, g_r, _ = _reference_step(ref, opt_r, crit, data.clone(), target, org)
            if dropin_bn:
                assert max(bn_err) <= TOL, (kind, step, "BatchNorm outputs", max(bn_err))
                bn_err.clear()
            dl = abs(float(lo) - float(lr_))
            assert dl <= TOL * max(1.0, abs(float(lr_))), (kind, step, "loss", float(lo), float(lr_))
            assert _rel(out_o, out_r) <= TOL, (kind, step, "log-probs", _rel(out_o, out_r))
            worst = 0.0
            for n in g_o:
                if n in FC_BIAS:
                    d = float((g_o[n].double() - g_r[n].double()).norm())
                    assert d <= TOL, (kind, step, n, "grad (abs)", d)
                    continue
                e = _rel(g_o[n], g_r[n])
                worst = max(worst, e)
                assert e <= TOL, (kind, step, n, "grad", e)
            named_o = dict(ours.module.named_parameters())
            named_r = dict(ref.module.named_parameters())
            if org:
                off_total, upd = 0, 0.0
                for n in BINARY_W:
                    a, b = named_o[n].org, named_r[n].org
                    # the .org protocol under DDP: the latent took torch's Adam step on the all-reduced
                    # gradient and the clamp -- float64 Adam from the pre-step latent and moments
                    p0, st = pre_o[n]
                    t = int(st.get("step", 0)) + 1
                    g64 = g_o[n].double()
                    m = (st["exp_avg"].double() if "exp_avg" in st else torch.zeros_like(g64)) * 0.9 + 0.1 * g64
                    v = (st["exp_avg_sq"].double() if "exp_avg_sq" in st else torch.zeros_like(g64)) * 0.999 \
                        + 0.001 * g64 * g64
                    want = p0.double() - (LR / (1 - 0.9 ** t)) * m / (v.sqrt() / (1 - 0.999 ** t) ** 0.5 + 1e-8)
                    d = float((a.double() - want.clamp(-1, 1)).abs().max())
                    upd = max(upd, d)
                    assert d <= 1e-6, (kind, step, n, "latent update != Adam + clamp of the DDP gradient", d)
                    assert float(a.abs().max()) <= 1.0
                    # the oracle's own update lands elsewhere only where Adam's lr * g / (|g| + eps)
                    # turns the gradients' rounding difference (checked above) into a step change
                    off_total += int(((a - b).abs() > 1e-6).sum())
                report.append(f"step {step}: loss {float(lo):.6f} |d| {dl:.2e}, worst grad {worst:.2e}, "
                              f"update vs float64 Adam {upd:.1e}, latents off the oracle's own update "
                              f"{off_total}")
            else:
                for n in ("bn1.weight", "bn1.bias", "bn2.weight", "bn2.bias", "bn3.weight", "bn3.bias",
                          "fc4.weight", "fc4.bias"):
                    e = _rel(named_o[n].data, named_r[n].data)
                    assert e <= TOL, (kind, step, n, "param", e)
                for n in BINARY_W:                 # frozen at the initial signs on both sides
                    assert torch.equal(named_o[n].org.sign(), named_r[n].org.sign()), (kind, step, n)
                report.append(f"step {step}: loss {float(lo):.6f} |d| {dl:.2e}, worst grad {worst:.2e}")
        params = [p.detach().cpu().numpy() for p in ours.module.parameters()]
        orgs = [p.org.detach().cpu().numpy() for p in ours.module.parameters() if hasattr(p, "org")]
        q.put((rank, {"params": params, "orgs": orgs, "report": report}))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


@pytest.mark.parametrize("kind", ["org", "frozen", "org-bn"])
def test_ddp_around_dropin_modules_matches_reference_semantics(kind):
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
    for line in out[0]["report"]:
        print(f"[{kind}] {line}")
    for a, b in zip(out[0]["params"] + out[0]["orgs"], out[1]["params"] + out[1]["orgs"]):
        np.testing.assert_array_equal(a, b)       # DDP kept the replicas identical
